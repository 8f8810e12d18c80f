// sh_aggregation.cpp — incremental `define aggregation ... every sec...year` roll-ups.
#include "sh_runtime.h"

struct sh_aggregation {};

extern "C" int sh_aggregation_create(sh_ctx* ctx, const sh_aggregation_desc* desc, sh_aggregation** out) {
    (void)ctx; (void)desc; (void)out;
    return sh_fail(SH_ERR_UNSUPPORTED, "incremental aggregation not yet on the GPU");
}
extern "C" int sh_aggregation_destroy(sh_aggregation* a) { delete a; return SH_OK; }
extern "C" int sh_aggregation_push(sh_aggregation* a, const sh_batch* b) {
    (void)a; (void)b;
    return sh_fail(SH_ERR_UNSUPPORTED, "incremental aggregation not yet on the GPU");
}
extern "C" int sh_aggregation_push_device(sh_aggregation* a, const sh_batch* b) {
    (void)a; (void)b;
    return sh_fail(SH_ERR_UNSUPPORTED, "incremental aggregation not yet on the GPU");
}
extern "C" int sh_aggregation_advance_time(sh_aggregation* a, int64_t now) {
    (void)a; (void)now;
    return sh_fail(SH_ERR_UNSUPPORTED, "incremental aggregation not yet on the GPU");
}
extern "C" int sh_aggregation_table(sh_aggregation* a, int32_t duration, const sh_out** out) {
    (void)a; (void)duration; (void)out;
    return sh_fail(SH_ERR_UNSUPPORTED, "incremental aggregation not yet on the GPU");
}
