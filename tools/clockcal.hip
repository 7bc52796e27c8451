// tools/clockcal.hip -- calibrates the two in-kernel counters against HIP
// events: s_memrealtime (wall clock) and s_memtime (shader clock), so that
// clock probes inside the AES kernels (CYAES_CLOCK_PROBE) can be read in
// seconds and GHz.  One wave per CU spins on s_memrealtime for a fixed tick
// count; the event time gives the tick rate.
// build: hipcc -O3 --offload-arch=gfx950 tools/clockcal.hip -o build/clockcal
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void spin(uint64_t ticks, unsigned long long* out) {
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime(), t0 = __builtin_amdgcn_s_memtime();
    uint64_t r = r0;
    while (r - r0 < ticks) r = __builtin_amdgcn_s_memrealtime();
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        out[0] = r - r0;
        out[1] = t1 - t0;
    }
}

int main() {
    int wall_khz = 0, clk_khz = 0;
    CK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
    CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
    unsigned long long* d;
    CK(hipMalloc(&d, 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    spin<<<256, 64>>>(1000, d);
    CK(hipDeviceSynchronize());
    for (uint64_t ticks : {1000000ull, 5000000ull}) {
        CK(hipEventRecord(e0));
        spin<<<256, 64>>>(ticks, d);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned long long h[2];
        CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
        printf("{\"ticks\": %llu, \"event_ms\": %.3f, \"realtime_mhz\": %.2f, \"memtime_per_realtime\": %.4f, "
               "\"attr_wallclock_khz\": %d, \"attr_clock_khz\": %d}\n",
               h[0], ms, h[0] / (ms * 1e3), (double)h[1] / (double)h[0], wall_khz, clk_khz);
    }
    return 0;
}
