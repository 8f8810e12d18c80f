// sh_sliding.cpp — sliding `#window.time(T)` group-by queries (TimeWindowProcessor semantics).
#include "sh_runtime.h"

struct SlidingImpl {};

int sliding_create(sh_query* q) {
    (void)q;
    return sh_fail(SH_ERR_UNSUPPORTED, "sliding time window not yet on the GPU");
}
int sliding_push(sh_query* q, const sh_batch* b, bool host_out, const sh_out** out) {
    (void)q; (void)b; (void)host_out; (void)out;
    return sh_fail(SH_ERR_UNSUPPORTED, "sliding time window not yet on the GPU");
}
int sliding_advance(sh_query* q, int64_t now, const sh_out** out) {
    (void)q; (void)now; (void)out;
    return sh_fail(SH_ERR_UNSUPPORTED, "sliding time window not yet on the GPU");
}
void sliding_destroy(sh_query* q) { (void)q; }
