// tools/valurate.hip -- issue rate of single VALU instructions on gfx950
// (wave64 lane-ops per clk per CU), by op and waves per SIMD.  Inline asm so
// the compiler cannot fuse or drop the ops; 8 independent chains per wave.
// Answers: do the integer ops the AES rounds use (v_perm_b32, v_bitop3_b32,
// v_xor_b32, v_lshl_or_b32) issue at the SIMD-32 rate (2 cycles per wave64
// instruction, as v_fma_f32) or at half of it?
// Build: hipcc -O3 --offload-arch=gfx950 tools/valurate.hip -o build/valurate
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

#define OP8(ins)                                                                                            \
    asm volatile(ins " %0, %0, %8\n\t" ins " %1, %1, %8\n\t" ins " %2, %2, %8\n\t" ins " %3, %3, %8\n\t" ins \
                     " %4, %4, %8\n\t" ins " %5, %5, %8\n\t" ins " %6, %6, %8\n\t" ins " %7, %7, %8"         \
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) \
                 : "v"(y))
#define OP8_SDWA(ins)                                                                                        \
    asm volatile(ins "\n\t" ins "\n\t" ins "\n\t" ins "\n\t" ins "\n\t" ins "\n\t" ins "\n\t" ins \
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) \
                 : "v"(y))
#define OP8_3(ins, suf)                                                                                        \
    asm volatile(ins " %0, %0, %8, %9" suf "\n\t" ins " %1, %1, %8, %9" suf "\n\t" ins " %2, %2, %8, %9" suf        \
                     "\n\t" ins " %3, %3, %8, %9" suf "\n\t" ins " %4, %4, %8, %9" suf "\n\t" ins " %5, %5, %8, %9" \
                     suf "\n\t" ins " %6, %6, %8, %9" suf "\n\t" ins " %7, %7, %8, %9" suf                         \
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) \
                 : "v"(y), "v"(z))

template <int OP>
__global__ __launch_bounds__(1024, 1) void k(uint32_t* out, int iters, unsigned long long* clk) {
    __shared__ uint32_t pin[24576];  // 96 KiB: one workgroup per CU
    if (iters < 0) pin[threadIdx.x] = 1;
    uint32_t x[8];
#pragma unroll
    for (int j = 0; j < 8; j++) x[j] = threadIdx.x * 31u + j;
    const uint32_t y = blockIdx.x * 3u + 1, z = threadIdx.x ^ 0x5555u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            if (OP == 0) OP8("v_xor_b32");
            if (OP == 1) OP8("v_add_u32");
            if (OP == 2) OP8_3("v_perm_b32", "");
            if (OP == 3) OP8_3("v_bitop3_b32", " bitop3:0x96");
            if (OP == 4) OP8_3("v_lshl_or_b32", "");
            if (OP == 5) OP8_3("v_fma_f32", "");
            if (OP == 6) OP8_3("v_add3_u32", "");
            if (OP == 7) OP8("v_and_b32");
            // address of an LDS row: byte k of a state word into byte 1, the
            // lane bits in bytes 0 and 2 preserved (no restore needed)
            if (OP == 8) {
                asm volatile(
                    "v_mov_b32_sdwa %0, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\n\t"
                    "v_mov_b32_sdwa %1, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2\n\t"
                    "v_mov_b32_sdwa %2, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3\n\t"
                    "v_mov_b32_sdwa %3, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1\n\t"
                    "v_mov_b32_sdwa %4, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\n\t"
                    "v_mov_b32_sdwa %5, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2\n\t"
                    "v_mov_b32_sdwa %6, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3\n\t"
                    "v_mov_b32_sdwa %7, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1"
                    : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
                    : "v"(y ^ x[u & 7]));
            }
            if (OP == 9) {  // v_or_b32_sdwa byte-select (what the compiler emits in merges)
                asm volatile(
                    "v_or_b32_sdwa %0, %0, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0\n\t"
                    "v_or_b32_sdwa %1, %1, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n\t"
                    "v_or_b32_sdwa %2, %2, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2\n\t"
                    "v_or_b32_sdwa %3, %3, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3\n\t"
                    "v_or_b32_sdwa %4, %4, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0\n\t"
                    "v_or_b32_sdwa %5, %5, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n\t"
                    "v_or_b32_sdwa %6, %6, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2\n\t"
                    "v_or_b32_sdwa %7, %7, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
                    : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
                    : "v"(y));
            }
            if (OP == 10) OP8_3("v_bfi_b32", "");
            if (OP == 11) OP8_3("v_and_or_b32", "");
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) acc ^= x[j];
    if (iters < 0) acc ^= pin[threadIdx.x ^ 1];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
        clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <int OP>
static void run(const char* name, int threads, int cus, uint32_t* d_out, unsigned long long* d_clk) {
    const int iters = 20000;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(k<OP>, dim3(cus), dim3(threads), 0, 0, d_out, iters / 10, d_clk);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(k<OP>, dim3(cus), dim3(threads), 0, 0, d_out, iters, d_clk);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    unsigned long long* h = (unsigned long long*)malloc(16ull * cus);
    CHECK(hipMemcpy(h, d_clk, 16ull * cus, hipMemcpyDeviceToHost));
    double cyc = 0, real = 0;
    for (int i = 0; i < cus; i++) {
        cyc += (double)h[2 * i];
        real += (double)h[2 * i + 1];
    }
    free(h);
    const double ghz = cyc / real * 0.1;
    const double ops = 64.0 * threads * iters;  // lane-ops per CU
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"clock_ghz\": %.3f, \"lane_ops_per_clk_cu\": %.2f}\n",
           name, threads / 256, ms, ghz, ops / (ms * 1e-3 * ghz * 1e9));
    fflush(stdout);
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t* d_out;
    unsigned long long* d_clk;
    CHECK(hipMalloc(&d_out, (size_t)cus * 1024 * 4));
    CHECK(hipMalloc(&d_clk, (size_t)cus * 16));
    for (int t : {256, 512, 1024}) {
        run<0>("v_xor_b32", t, cus, d_out, d_clk);
        run<1>("v_add_u32", t, cus, d_out, d_clk);
        run<2>("v_perm_b32", t, cus, d_out, d_clk);
        run<3>("v_bitop3_b32", t, cus, d_out, d_clk);
        run<4>("v_lshl_or_b32", t, cus, d_out, d_clk);
        run<5>("v_fma_f32", t, cus, d_out, d_clk);
        run<6>("v_add3_u32", t, cus, d_out, d_clk);
        run<7>("v_and_b32", t, cus, d_out, d_clk);
        run<8>("v_mov_b32_sdwa_preserve_plus_xor", t, cus, d_out, d_clk);
        run<9>("v_or_b32_sdwa", t, cus, d_out, d_clk);
        run<10>("v_bfi_b32", t, cus, d_out, d_clk);
        run<11>("v_and_or_b32", t, cus, d_out, d_clk);
    }
    return 0;
}
