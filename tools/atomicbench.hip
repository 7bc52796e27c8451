// tools/atomicbench.hip -- work-ticket atomics on MI355X: what one returning
// atomicAdd per wave costs when every wave of a persistent 256 x 1024 grid
// takes tickets from (a) one counter, (b) one counter per XCD, (c) one per
// workgroup, (d) one per wave, at agent and at workgroup scope.  Each wave
// takes `iters` tickets back to back (each address depends on the previous
// result, so they are serialised per wave), with `spin` dependent VALU ops
// between them.  Prints per mode: ns per ticket per wave and tickets/s over
// the grid.  (The dynamic decrypt ranges of r04 took one ticket per 2-step
// range from a single counter and ran 2x slower: this finds out why.)
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int MODE, bool WG_SCOPE>
__global__ __launch_bounds__(1024, 1) void k_tickets(unsigned* ctr, unsigned long long* sink, int iters, int spin) {
    const unsigned wave = blockIdx.x * 16 + (threadIdx.x >> 6);
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 15;
    unsigned slot = MODE == 0 ? 0 : MODE == 1 ? xcc : MODE == 2 ? blockIdx.x : wave;
    unsigned* p = ctr + 64 * slot;  // a 256-B line per counter
    unsigned acc = threadIdx.x;
    for (int i = 0; i < iters; i++) {
        unsigned t = 0;
        if ((threadIdx.x & 63) == 0) {
            if (WG_SCOPE)
                t = __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            else
                t = __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        t = __builtin_amdgcn_readfirstlane(t);
        acc += t;
        for (int s = 0; s < spin; s++) acc = acc * 1664525u + 1013904223u;
    }
    if (acc == 0x12345678u) sink[0] = acc;  // keep the work
}

template <int MODE, bool WG>
float run(unsigned* ctr, unsigned long long* sink, int iters, int spin) {
    hipMemset(ctr, 0, 64 * 4 * 8192);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_tickets<MODE, WG>), dim3(256), dim3(1024), 0, 0, ctr, sink, iters, spin);
    hipEventRecord(a);
    hipLaunchKernelGGL((k_tickets<MODE, WG>), dim3(256), dim3(1024), 0, 0, ctr, sink, iters, spin);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    unsigned* ctr;
    unsigned long long* sink;
    if (hipMalloc(&ctr, 64 * 4 * 8192) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) return 1;
    const char* names[4] = {"one counter", "per XCD", "per workgroup", "per wave"};
    for (int spin : {0, 2000}) {
        const int iters = 200;
        const float base = run<3, false>(ctr, sink, 0, spin) ;
        (void)base;
        float ms[2][4];
        ms[0][0] = run<0, false>(ctr, sink, iters, spin);
        ms[0][1] = run<1, false>(ctr, sink, iters, spin);
        ms[0][2] = run<2, false>(ctr, sink, iters, spin);
        ms[0][3] = run<3, false>(ctr, sink, iters, spin);
        ms[1][0] = run<0, true>(ctr, sink, iters, spin);
        ms[1][1] = run<1, true>(ctr, sink, iters, spin);
        ms[1][2] = run<2, true>(ctr, sink, iters, spin);
        ms[1][3] = run<3, true>(ctr, sink, iters, spin);
        const float nospin = run<3, false>(ctr, sink, iters, 0);
        (void)nospin;
        for (int sc = 0; sc < 2; sc++)
            for (int m = 0; m < 4; m++)
                printf("{\"mode\": \"%s\", \"scope\": \"%s\", \"spin\": %d, \"iters\": %d, \"ms\": %.3f, "
                       "\"ns_per_ticket_per_wave\": %.1f, \"Mtickets_per_s\": %.1f}\n",
                       names[m], sc ? "workgroup" : "agent", spin, iters, ms[sc][m], ms[sc][m] * 1e6 / iters,
                       4096.0 * iters / (ms[sc][m] * 1e3));
    }
    return 0;
}
