// tools/vbank.hip -- does v_bitop3_b32 issue slower when its three VGPR
// sources share a register bank (VGPR index mod 4)?  The bitsliced decrypt
// prototype (tools/bitslice.hip, removed in r04; git history) issues ~51 lane-ops/clk/CU where a
// v_bitop3_b32 microbench (tools/valurate.hip, sources in distinct banks)
// reached ~100.  Explicit VGPR numbers, 8 independent chains per wave,
// 16 waves/CU, in-kernel clock.
// build: hipcc -O3 --offload-arch=gfx950 tools/vbank.hip -o build/vbank
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

// dst chains v[40..47]; sources per pattern:
//  0 distinct banks: src0 = chain (bank 0..3 varies), src1 = v1 (bank 1), src2 = v2 (bank 2)
//  1 two sources same bank: src1 = v4, src2 = v8 (both bank 0)
//  2 all three same bank: chain regs v40,v44,.. (bank 0) with src1 v4 src2 v8
//  3 xor2 (VOP2 v_xor_b32) distinct banks
#define CL "v1", "v2", "v4", "v8", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v52", "v56", "v60"
template <int P>
__global__ __launch_bounds__(1024, 1) void k(uint32_t* out, int iters, unsigned long long* clk) {
    __shared__ uint32_t pin[24576];
    if (iters < 0) pin[threadIdx.x] = 1;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    asm volatile("v_mov_b32 v1, 0x1234\n\tv_mov_b32 v2, 0x5678\n\tv_mov_b32 v4, 0x9abc\n\tv_mov_b32 v8, 0xdef0\n\t"
                 "v_mov_b32 v40, 1\n\tv_mov_b32 v41, 2\n\tv_mov_b32 v42, 3\n\tv_mov_b32 v43, 4\n\t"
                 "v_mov_b32 v44, 5\n\tv_mov_b32 v45, 6\n\tv_mov_b32 v46, 7\n\tv_mov_b32 v47, 8\n\t"
                 "v_mov_b32 v48, 9\n\tv_mov_b32 v52, 10\n\tv_mov_b32 v56, 11\n\tv_mov_b32 v60, 12" ::: CL);
    for (int it = 0; it < iters; it++) {
        if (P == 0)
            asm volatile(
                "v_bitop3_b32 v40, v40, v1, v2 bitop3:0x96\n\tv_bitop3_b32 v41, v41, v1, v2 bitop3:0x96\n\t"
                "v_bitop3_b32 v42, v42, v1, v2 bitop3:0x96\n\tv_bitop3_b32 v43, v43, v1, v2 bitop3:0x96\n\t"
                "v_bitop3_b32 v45, v45, v1, v2 bitop3:0x96\n\tv_bitop3_b32 v46, v46, v1, v2 bitop3:0x96\n\t"
                "v_bitop3_b32 v47, v47, v1, v2 bitop3:0x96\n\tv_bitop3_b32 v44, v44, v1, v2 bitop3:0x96" ::: CL);
        if (P == 1)
            asm volatile(
                "v_bitop3_b32 v41, v41, v4, v8 bitop3:0x96\n\tv_bitop3_b32 v42, v42, v4, v8 bitop3:0x96\n\t"
                "v_bitop3_b32 v43, v43, v4, v8 bitop3:0x96\n\tv_bitop3_b32 v45, v45, v4, v8 bitop3:0x96\n\t"
                "v_bitop3_b32 v46, v46, v4, v8 bitop3:0x96\n\tv_bitop3_b32 v47, v47, v4, v8 bitop3:0x96\n\t"
                "v_bitop3_b32 v41, v41, v4, v8 bitop3:0x96\n\tv_bitop3_b32 v42, v42, v4, v8 bitop3:0x96" ::: CL);
        if (P == 2)
            asm volatile(
                "v_bitop3_b32 v40, v40, v4, v8 bitop3:0x96\n\tv_bitop3_b32 v44, v44, v4, v8 bitop3:0x96\n\t"
                "v_bitop3_b32 v48, v48, v4, v8 bitop3:0x96\n\tv_bitop3_b32 v52, v52, v4, v8 bitop3:0x96\n\t"
                "v_bitop3_b32 v56, v56, v4, v8 bitop3:0x96\n\tv_bitop3_b32 v60, v60, v4, v8 bitop3:0x96\n\t"
                "v_bitop3_b32 v40, v40, v4, v8 bitop3:0x96\n\tv_bitop3_b32 v44, v44, v4, v8 bitop3:0x96" ::: CL);
        if (P == 3)
            asm volatile(
                "v_xor_b32 v40, v40, v1\n\tv_xor_b32 v41, v41, v1\n\tv_xor_b32 v42, v42, v1\n\tv_xor_b32 v43, v43, v1\n\t"
                "v_xor_b32 v44, v44, v1\n\tv_xor_b32 v45, v45, v1\n\tv_xor_b32 v46, v46, v1\n\tv_xor_b32 v47, v47, v1" ::: CL);
        // 4: dependent chain of 8 (each reads the previous result): latency
        if (P == 4)
            asm volatile(
                "v_bitop3_b32 v40, v40, v1, v2 bitop3:0x96\n\tv_bitop3_b32 v40, v40, v1, v2 bitop3:0x96\n\t"
                "v_bitop3_b32 v40, v40, v1, v2 bitop3:0x96\n\tv_bitop3_b32 v40, v40, v1, v2 bitop3:0x96\n\t"
                "v_bitop3_b32 v40, v40, v1, v2 bitop3:0x96\n\tv_bitop3_b32 v40, v40, v1, v2 bitop3:0x96\n\t"
                "v_bitop3_b32 v40, v40, v1, v2 bitop3:0x96\n\tv_bitop3_b32 v40, v40, v1, v2 bitop3:0x96" ::: CL);
        // 5: independent, but each instruction's sources are the two previous results (distinct banks)
        if (P == 5)
            asm volatile(
                "v_bitop3_b32 v40, v41, v42, v43 bitop3:0x96\n\tv_bitop3_b32 v45, v46, v47, v44 bitop3:0x96\n\t"
                "v_bitop3_b32 v41, v42, v43, v40 bitop3:0x96\n\tv_bitop3_b32 v46, v47, v44, v45 bitop3:0x96\n\t"
                "v_bitop3_b32 v42, v43, v40, v41 bitop3:0x96\n\tv_bitop3_b32 v47, v44, v45, v46 bitop3:0x96\n\t"
                "v_bitop3_b32 v43, v40, v41, v42 bitop3:0x96\n\tv_bitop3_b32 v44, v45, v46, v47 bitop3:0x96" ::: CL);
    }
    uint32_t r;
    asm volatile("v_mov_b32 %0, v40" : "=v"(r) :: CL);
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (r == 0x12345u) out[0] = r;
    if (threadIdx.x == 0) {
        atomicAdd(&clk[0], t1 - t0);
        atomicAdd(&clk[1], r1 - r0);
    }
}

template <int P>
void run(const char* name, int cus, uint32_t* d_out, unsigned long long* d_clk) {
    const int iters = 20000;
    CHECK(hipMemset(d_clk, 0, 16));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(k<P>, dim3(cus), dim3(1024), 0, 0, d_out, iters, d_clk);
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(k<P>, dim3(cus), dim3(1024), 0, 0, d_out, iters, d_clk);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    CHECK(hipMemset(d_clk, 0, 16));
    hipLaunchKernelGGL(k<P>, dim3(cus), dim3(1024), 0, 0, d_out, iters, d_clk);
    CHECK(hipDeviceSynchronize());
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    unsigned long long c[2];
    CHECK(hipMemcpy(c, d_clk, 16, hipMemcpyDeviceToHost));
    const double ghz = (double)c[0] / c[1] * 0.1;
    const double ops = (double)cus * 1024 * iters * 8;
    printf("{\"test\": \"%s\", \"ms\": %.3f, \"clock_ghz\": %.3f, \"lane_ops_per_clk_cu\": %.2f}\n", name, ms, ghz,
           ops / (ms * 1e-3) / (ghz * 1e9) / cus);
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    uint32_t* d_out;
    unsigned long long* d_clk;
    CHECK(hipMalloc(&d_out, 64));
    CHECK(hipMalloc(&d_clk, 16));
    run<0>("bitop3 distinct banks", p.multiProcessorCount, d_out, d_clk);
    run<1>("bitop3 src1,src2 same bank", p.multiProcessorCount, d_out, d_clk);
    run<2>("bitop3 all three same bank", p.multiProcessorCount, d_out, d_clk);
    run<3>("v_xor_b32", p.multiProcessorCount, d_out, d_clk);
    run<4>("bitop3 dependent chain", p.multiProcessorCount, d_out, d_clk);
    run<5>("bitop3 sources = recent results", p.multiProcessorCount, d_out, d_clk);
    return 0;
}
