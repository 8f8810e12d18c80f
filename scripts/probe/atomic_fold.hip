// probe: cost of folding the C2 stream (2^25 events, 1000 per ms, timeBatch(1 sec), 100k uniform keys) by
// device atomics into a per-(window, key) table instead of the exact path's multisplit + ordered fold.
// Decides whether a tolerance mode (double sums in any order) could beat the exact 1.06 ms step:
// the atomics alone must cost well under it. Variants: the stream read alone; count + sum; count + sum +
// min + max + first-occurrence index (what a flush needs).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int kKeys = 100000;
constexpr int kPerWindow = 1000000;  // 1000 events per ms x 1000 ms

__device__ inline uint64_t ordered(double d) {
    const uint64_t b = __double_as_longlong(d);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

template <int kMode>
__global__ __launch_bounds__(256) void k_fold(const int64_t* __restrict__ ts, const uint32_t* __restrict__ key,
                                              const double* __restrict__ v, int64_t n, uint32_t* cnt, double* sum,
                                              unsigned long long* mn, unsigned long long* mx, uint32_t* first,
                                              double* sink) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t w = ts[i] / kPerWindow;
    const uint32_t k = key[i];
    const double x = v[i];
    if (kMode == 0) {
        if (x == -1.0 && k == 7u && w == -3) sink[0] = x;  // keeps the loads live
        return;
    }
    const int64_t s = w * kKeys + k;
    atomicAdd(cnt + s, 1u);
    unsafeAtomicAdd(sum + s, x);
    if (kMode == 2) {
        const unsigned long long o = ordered(x);
        atomicMin(mn + s, o);
        atomicMax(mx + s, o);
        atomicMin(first + s, (uint32_t)(i - w * kPerWindow));
    }
}

int main() {
    CK(hipSetDevice(0));
    const int64_t n = 1ll << 25;
    const int64_t nw = n / kPerWindow + 2;
    std::vector<int64_t> hts(n);
    std::vector<uint32_t> hk(n);
    std::vector<double> hv(n);
    uint64_t r = 0x9E3779B97F4A7C15ull;
    for (int64_t i = 0; i < n; i++) {
        r ^= r << 13; r ^= r >> 7; r ^= r << 17;
        hts[i] = i;
        hk[i] = (uint32_t)(r % kKeys);
        hv[i] = (double)((r >> 20) % 100000) / 8.0;
    }
    int64_t* ts; uint32_t* key; double* v; uint32_t* cnt; double* sum; unsigned long long* mn; unsigned long long* mx;
    uint32_t* first; double* sink;
    const size_t slots = (size_t)nw * kKeys;
    CK(hipMalloc(&ts, n * 8)); CK(hipMalloc(&key, n * 4)); CK(hipMalloc(&v, n * 8));
    CK(hipMalloc(&cnt, slots * 4)); CK(hipMalloc(&sum, slots * 8)); CK(hipMalloc(&mn, slots * 8));
    CK(hipMalloc(&mx, slots * 8)); CK(hipMalloc(&first, slots * 4)); CK(hipMalloc(&sink, 8));
    CK(hipMemcpy(ts, hts.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(key, hk.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(v, hv.data(), n * 8, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const dim3 grid((unsigned)((n + 255) / 256));
    const char* names[3] = {"stream read only (20 B/event)", "count + sum atomics", "count + sum + min + max + first atomics"};
    for (int mode = 0; mode < 3; mode++) {
        float best = 1e30f, total = 0.f;
        const int reps = 10;
        for (int rep = 0; rep < reps + 2; rep++) {
            CK(hipMemset(cnt, 0, slots * 4)); CK(hipMemset(sum, 0, slots * 8));
            CK(hipMemset(mn, 0xFF, slots * 8)); CK(hipMemset(mx, 0, slots * 8)); CK(hipMemset(first, 0xFF, slots * 4));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            if (mode == 0) hipLaunchKernelGGL(k_fold<0>, grid, dim3(256), 0, 0, ts, key, v, n, cnt, sum, mn, mx, first, sink);
            if (mode == 1) hipLaunchKernelGGL(k_fold<1>, grid, dim3(256), 0, 0, ts, key, v, n, cnt, sum, mn, mx, first, sink);
            if (mode == 2) hipLaunchKernelGGL(k_fold<2>, grid, dim3(256), 0, 0, ts, key, v, n, cnt, sum, mn, mx, first, sink);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep >= 2) { total += ms; if (ms < best) best = ms; }
        }
        printf("%-42s  mean %.3f ms  best %.3f ms  %.2f G atomic-events/s\n", names[mode], total / reps, best,
               n / (best * 1e6));
    }
    std::vector<uint32_t> hc(slots);
    CK(hipMemcpy(hc.data(), cnt, slots * 4, hipMemcpyDeviceToHost));
    uint64_t tot = 0;
    for (size_t i = 0; i < slots; i++) tot += hc[i];
    printf("check: counted %llu of %lld events\n", (unsigned long long)tot, (long long)n);
    return 0;
}
