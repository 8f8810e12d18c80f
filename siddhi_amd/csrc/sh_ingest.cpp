// sh_ingest.cpp — double-buffered host ingest (north_star: "The Java host code packs ComplexEventChunk
// micro-batches into pinned columnar SoA buffers ... with double-buffered hipMemcpyAsync on side
// streams").
//
// The reference hands each InputHandler.send(Event[]) to the junction and returns
// (InputHandler.java:85-96, StreamJunction.sendEvent :104-131; with @async the disruptor batches
// events for the processing thread, :279-316). Here the host side stages micro-batch i+1 into one
// of two device slots on the context's copy stream while micro-batch i is processed on the compute
// stream: sh_stage queues the H2D copies and returns, sh_push_staged makes the compute stream wait
// for that slot's copy, runs the push and records when the slot's device buffers are free again.
#include <hip/hip_runtime.h>

#include <string>

#include "sh_runtime.h"

#define HIPCHK(x)                                                                                          \
    do {                                                                                                   \
        hipError_t _e = (x);                                                                               \
        if (_e != hipSuccess) return sh_fail(SH_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(_e)); \
    } while (0)
#define RCHK(x)            \
    do {                   \
        int _r = (x);      \
        if (_r) return _r; \
    } while (0)

static int ingest_init(sh_query* q) {
    auto& g = q->ing;
    for (int i = 0; i < 2; i++) {
        if (g.copied[i]) continue;
        HIPCHK(hipEventCreateWithFlags(&g.copied[i], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&g.consumed[i], hipEventDisableTiming));
        HIPCHK(hipEventCreate(&g.c0[i]));
        HIPCHK(hipEventCreate(&g.c1[i]));
    }
    return SH_OK;
}

void ingest_destroy(sh_query* q) {
    auto& g = q->ing;
    for (int i = 0; i < 2; i++) {
        hipEvent_t evs[] = {g.copied[i], g.consumed[i], g.c0[i], g.c1[i]};
        for (auto e : evs) if (e) (void)hipEventDestroy(e);
        g.copied[i] = g.consumed[i] = g.c0[i] = g.c1[i] = nullptr;
    }
}

extern "C" int sh_stage(sh_query* q, const sh_batch* b, int32_t* ticket) {
    SH_RANGE("sh_stage");
    if (!q || !b || !ticket) return sh_fail(SH_ERR_INVALID, "sh_stage: NULL argument");
    if (b->n < 0) return sh_fail(SH_ERR_INVALID, "negative batch size");
    if (b->n > 0 && !b->ts) return sh_fail(SH_ERR_INVALID, "batch without timestamps");
    RCHK(check_batch_cols(q, b));
    if (q->wide) return sh_fail(SH_ERR_UNSUPPORTED, "queries with wide group keys take sh_push / sh_push_device");
    auto& g = q->ing;
    if (g.outstanding >= 2) return sh_fail(SH_ERR_INVALID, "sh_stage: two staged batches are waiting for sh_push_staged");
    RCHK(ingest_init(q));
    const int slot = g.next_stage;
    // a small batch in pinned host memory that the small-push kernel can take: no copy at all, the
    // kernel reads it over PCIe in place (hipHostGetDevicePointer refuses pageable memory)
    g.zc[slot] = false;
    if (query_small_eligible(q, b->n)) {
        sh_batch dv = *b;
        bool ok = hipHostGetDevicePointer((void**)&dv.ts, (void*)b->ts, 0) == hipSuccess;
        for (int c = 0; c < q->d.n_cols && ok; c++)
            if (b->cols[c]) ok = hipHostGetDevicePointer((void**)&dv.cols[c], (void*)b->cols[c], 0) == hipSuccess;
        (void)hipGetLastError();
        if (ok) {
            g.zc[slot] = true;
            g.host[slot] = *b;
            g.dev[slot] = dv;
            g.bytes[slot] = 0;
            g.ticket_gen[slot] = ++g.gen;
            g.next_stage ^= 1;
            g.outstanding++;
            *ticket = (int32_t)((g.ticket_gen[slot] << 1) | (uint32_t)slot);
            return SH_OK;
        }
    }
    hipStream_t cs = q->ctx->copy_stream;
    // the slot's previous batch must have been consumed by its push before it is overwritten
    if (g.used[slot]) HIPCHK(hipStreamWaitEvent(cs, g.consumed[slot], 0));
    // slot growth allocates outside stream order (hipMalloc): the copy stream may not depend on an
    // allocation queued on the compute stream
    {
        StreamScope none(nullptr);
        sh_batch dev;
        HIPCHK(hipEventRecord(g.c0[slot], cs));
        RCHK(g.slot[slot].stage(cs, b, q->d.n_cols, q->d.col_types, &dev));
        HIPCHK(hipEventRecord(g.c1[slot], cs));
        g.dev[slot] = dev;
    }
    HIPCHK(hipEventRecord(g.copied[slot], cs));
    int64_t bytes = b->ts ? b->n * 8 : 0;
    for (int c = 0; c < q->d.n_cols; c++) if (b->cols[c]) bytes += b->n * (int64_t)type_size(q->d.col_types[c]);
    g.bytes[slot] = bytes;
    g.used[slot] = true;
    g.ticket_gen[slot] = ++g.gen;
    g.next_stage ^= 1;
    g.outstanding++;
    *ticket = (int32_t)((g.ticket_gen[slot] << 1) | (uint32_t)slot);
    return SH_OK;
}

extern "C" int sh_push_staged(sh_query* q, int32_t ticket, const sh_out** out) {
    SH_RANGE("sh_push_staged");
    StreamScope _ss(q && q->ctx ? q->ctx->stream : nullptr);
    if (!q || !out) return sh_fail(SH_ERR_INVALID, "sh_push_staged: NULL argument");
    auto& g = q->ing;
    const int slot = ticket & 1;
    if (g.outstanding == 0 || slot != g.next_push || (uint32_t)ticket >> 1 != g.ticket_gen[slot])
        return sh_fail(SH_ERR_INVALID, "sh_push_staged: tickets are pushed once, in the order they were staged");
    hipStream_t s = q->ctx->stream;
    g.outstanding--;
    g.next_push ^= 1;
    if (g.zc[slot]) {
        // read in place; staged on this stream only if the push leaves the small-push path
        q->zc_host = &g.host[slot];
        const int rc = query_push_staged(q, &g.dev[slot], out);
        q->zc_host = nullptr;
        g.last_h2d_ms = 0;
        g.last_h2d_bytes = 0;
        return rc;
    }
    HIPCHK(hipStreamWaitEvent(s, g.copied[slot], 0));
    const int rc = query_push_staged(q, &g.dev[slot], out);
    // the slot is free for the next sh_stage once the kernels that read it have run
    HIPCHK(hipEventRecord(g.consumed[slot], s));
    if (rc) return rc;
    float ms = 0;
    if (hipEventElapsedTime(&ms, g.c0[slot], g.c1[slot]) == hipSuccess) g.last_h2d_ms = ms;
    g.last_h2d_bytes = g.bytes[slot];
    return SH_OK;
}

extern "C" int sh_ingest_stats(sh_query* q, double* h2d_ms, int64_t* h2d_bytes) {
    if (!q || !h2d_ms || !h2d_bytes) return sh_fail(SH_ERR_INVALID, "sh_ingest_stats: NULL argument");
    *h2d_ms = q->ing.last_h2d_ms;
    *h2d_bytes = q->ing.last_h2d_bytes;
    return SH_OK;
}
