// Probe: do lanes of one wave that hit the same LDS counter in one ds_add_rtn get their returns in
// lane order? (The aggregation's ranking repairs the order either way; this measures how often it
// has to.) Build: hipcc -O3 --offload-arch=gfx950 lds_atomic_order.hip -o /tmp/lds_order
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ void probe(int M, int iters, unsigned long long* viol, unsigned long long* pairs) {
    __shared__ uint32_t cnt[4][1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned long long v = 0, p = 0;
    for (int it = 0; it < iters; it++) {
        for (int i = lane; i < 1024; i += 64) cnt[w][i] = 0;
        __builtin_amdgcn_wave_barrier();
        const uint32_t key = mix(blockIdx.x * 7919u + it * 104729u + w * 31u + lane) % (uint32_t)M;
        const uint32_t r = atomicAdd(&cnt[w][key], 1u);
        // compare with every lower lane holding the same key
        for (int j = 0; j < 64; j++) {
            const uint32_t kj = __shfl(key, j, 64), rj = __shfl(r, j, 64);
            if (j < lane && kj == key) { p++; if (rj > r) v++; }
        }
        __builtin_amdgcn_wave_barrier();
    }
    atomicAdd(viol, v);
    atomicAdd(pairs, p);
}

int main() {
    unsigned long long *d, h[2];
    hipMalloc(&d, 16);
    const int Ms[] = {1, 2, 7, 64, 390, 1000};
    for (int M : Ms) {
        hipMemset(d, 0, 16);
        hipLaunchKernelGGL(probe, dim3(2048), dim3(256), 0, 0, M, 64, d, d + 1);
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("M=%d same-key lane pairs=%llu out-of-lane-order=%llu\n", M, h[1], h[0]);
    }
    return 0;
}
