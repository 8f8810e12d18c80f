// probe: host time of hipMalloc vs virtual-memory mapping (hipMemCreate + hipMemMap + hipMemSetAccess)
// for buffers of 64 MB .. 1 GB on one MI355X (decides how a growing aggregation table should grow)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    for (size_t mb : {64, 256, 512, 1024}) {
        void* p = nullptr;
        double t0 = now_us();
        CK(hipMalloc(&p, mb << 20));
        double t1 = now_us();
        CK(hipMemset(p, 0, 16));
        CK(hipDeviceSynchronize());
        double t2 = now_us();
        CK(hipFree(p));
        double t3 = now_us();
        printf("hipMalloc %4zu MB: %8.1f us  first touch %8.1f us  hipFree %8.1f us\n", mb, t1 - t0, t2 - t1, t3 - t2);
    }
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    printf("granularity %zu\n", gran);
    hipDeviceptr_t base = nullptr;
    const size_t va = (size_t)16 << 30;
    CK(hipMemAddressReserve((void**)&base, va, 0, nullptr, 0));
    size_t mapped = 0;
    for (size_t mb : {64, 256, 512, 1024}) {
        const size_t sz = mb << 20;
        double t0 = now_us();
        hipMemGenericAllocationHandle_t h;
        CK(hipMemCreate(&h, sz, &prop, 0));
        CK(hipMemMap((char*)base + mapped, sz, 0, h, 0));
        hipMemAccessDesc acc = {};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        CK(hipMemSetAccess((char*)base + mapped, sz, &acc, 1));
        double t1 = now_us();
        CK(hipMemset((char*)base + mapped, 0, 16));
        CK(hipDeviceSynchronize());
        double t2 = now_us();
        printf("vmm map   %4zu MB: %8.1f us  first touch %8.1f us\n", mb, t1 - t0, t2 - t1);
        mapped += sz;
    }
    return 0;
}
