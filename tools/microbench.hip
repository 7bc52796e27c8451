// tools/microbench.hip -- gfx950 ceilings for the T-table AES inner loop.
//
// Measures, on the shapes the AES kernels use (16 waves per CU):
//   * conflict-free ds_read_b32 gather rate (lookups / clk / CU),
//   * VALU issue cost of the ops the round uses (v_perm, v_bitop3, v_alignbit),
//   * the mixed LDS + VALU rate at the round's ratio (VALU ops per lookup),
//   * the shader clock under that load (s_memtime vs s_memrealtime).
// Output: one JSON object per line.  Build: make microbench.
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

struct Clk {
    unsigned long long t0, t1, r0, r1;
};

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// LDS gathers: 16 independent conflict-free lookups per iteration, addresses
// derived from the previous iteration's values with one v_perm each (the AES
// pattern), plus EXTRA additional VALU ops per lookup.
template <int EXTRA>
__global__ __launch_bounds__(1024, 1) void k_lds(uint32_t* out, int iters, Clk* clk) {
    __shared__ uint32_t lds[24576];  // 96 KiB: one workgroup per CU
    for (int i = threadIdx.x; i < 24576; i += blockDim.x) lds[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t lo = (threadIdx.x & 31u) << 2;
    uint32_t s[16];
#pragma unroll
    for (int j = 0; j < 16; j++) s[j] = (threadIdx.x * 7919u + j * 104729u) | 1;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int it = 0; it < iters; it++) {
        uint32_t v[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint32_t a = __builtin_amdgcn_perm(s[j], lo, 0x0C0C0400u + ((j & 3) << 8));
            v[j] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + a);
        }
#pragma unroll
        for (int j = 0; j < 16; j++) {
            uint32_t x = v[j];
#pragma unroll
            for (int e = 0; e < EXTRA; e++) x = xor3(x, s[(j + 1 + e) & 15], 0x9e3779b9u);
            s[j] ^= x;
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) acc ^= s[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) {
        clk[blockIdx.x].t0 = t0;
        clk[blockIdx.x].r0 = r0;
        clk[blockIdx.x].t1 = __builtin_amdgcn_s_memtime();
        clk[blockIdx.x].r1 = __builtin_amdgcn_s_memrealtime();
    }
}

// Mixed gathers: per iteration 16 lookups, NV of them from a 1 KiB table in
// global memory (L1/L2 resident, SDWA byte-select address), the rest from LDS.
template <int NV>
__global__ __launch_bounds__(1024, 1) void k_mix(uint32_t* out, int iters, Clk* clk, const uint32_t* __restrict__ gtab) {
    __shared__ uint32_t lds[24576];  // 96 KiB: one workgroup per CU
    for (int i = threadIdx.x; i < 24576; i += blockDim.x) lds[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t lo = (threadIdx.x & 31u) << 2;
    uint32_t s[16];
#pragma unroll
    for (int j = 0; j < 16; j++) s[j] = (threadIdx.x * 7919u + j * 104729u) | 1;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int it = 0; it < iters; it++) {
        uint32_t v[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            if (j < NV) {
                v[j] = gtab[(s[j] >> (8 * (j & 3))) & 0xFF];
            } else {
                const uint32_t a = __builtin_amdgcn_perm(s[j], lo, 0x0C0C0400u + ((j & 3) << 8));
                v[j] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + a);
            }
        }
#pragma unroll
        for (int j = 0; j < 16; j++) s[j] ^= v[j];
    }
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) acc ^= s[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) {
        clk[blockIdx.x].t0 = t0;
        clk[blockIdx.x].r0 = r0;
        clk[blockIdx.x].t1 = __builtin_amdgcn_s_memtime();
        clk[blockIdx.x].r1 = __builtin_amdgcn_s_memrealtime();
    }
}

// Independent VMEM gathers beside the LDS stream: per
// iteration the 16 LDS chains of k_lds<0>, plus NV gathers from a 1 KiB
// global table whose addresses come from the LDS chains' state and whose
// results feed only an accumulator -- never an address, as the decrypt's
// last-round Si lookups feed only the store (cyr_rijndael.cpp:753-773).  DIST
// 0: consumed at the end of the iteration that issued them; 1: one iteration
// later.  If the TA path runs in parallel with the LDS, the LDS lookup rate
// stays at k_lds<0>'s while NV extra lookups per 16 ride along.
template <int NV, int DIST>
__global__ __launch_bounds__(1024, 1) void k_vmix(uint32_t* out, int iters, Clk* clk, const uint32_t* __restrict__ gtab) {
    __shared__ uint32_t lds[24576];  // 96 KiB: one workgroup per CU
    for (int i = threadIdx.x; i < 24576; i += blockDim.x) lds[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t lo = (threadIdx.x & 31u) << 2;
    uint32_t s[16];
#pragma unroll
    for (int j = 0; j < 16; j++) s[j] = (threadIdx.x * 7919u + j * 104729u) | 1;
    uint32_t acc = 0, held[NV > 0 ? NV : 1] = {};
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int it = 0; it < iters; it++) {
        uint32_t vv[NV > 0 ? NV : 1];
#pragma unroll
        for (int k = 0; k < NV; k++) vv[k] = gtab[(s[k] >> (8 * (k & 3))) & 0xFF];
        uint32_t v[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint32_t a = __builtin_amdgcn_perm(s[j], lo, 0x0C0C0400u + ((j & 3) << 8));
            v[j] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + a);
        }
#pragma unroll
        for (int j = 0; j < 16; j++) s[j] ^= v[j];
#pragma unroll
        for (int k = 0; k < NV; k++) {
            if (DIST == 0) acc ^= vv[k];
            else {
                acc ^= held[k];
                held[k] = vv[k];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < NV; k++) acc ^= held[k];
#pragma unroll
    for (int j = 0; j < 16; j++) acc ^= s[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) {
        clk[blockIdx.x].t0 = t0;
        clk[blockIdx.x].r0 = r0;
        clk[blockIdx.x].t1 = __builtin_amdgcn_s_memtime();
        clk[blockIdx.x].r1 = __builtin_amdgcn_s_memrealtime();
    }
}

// LDS peak: one v_perm per 4 conflict-free ds_read_b32 (offsets 0/64/128/192)
// and one xor3 per 2 reads, so VALU cannot bind.  B64: ds_read_b64 instead.
template <bool B64>
__global__ __launch_bounds__(1024, 1) void k_ldspeak(uint32_t* out, int iters, Clk* clk) {
    __shared__ uint32_t lds[24576];  // 96 KiB: one workgroup per CU
    for (int i = threadIdx.x; i < 24576; i += blockDim.x) lds[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t lo = (threadIdx.x & 31u) << (B64 ? 3 : 2);
    uint32_t s[4];
#pragma unroll
    for (int j = 0; j < 4; j++) s[j] = (threadIdx.x * 7919u + j * 104729u) | 1;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    const char* base = reinterpret_cast<const char*>(lds);
    for (int it = 0; it < iters; it++) {
        uint32_t a[4];
#pragma unroll
        for (int j = 0; j < 4; j++) a[j] = __builtin_amdgcn_perm(s[j], lo, 0x0C0C0400u + (j << 8));
        if (B64) {
            uint2 v[8];
            asm volatile(
                "ds_read_b64 %0, %8\n\tds_read_b64 %1, %8 offset:256\n\t"
                "ds_read_b64 %2, %9\n\tds_read_b64 %3, %9 offset:256\n\t"
                "ds_read_b64 %4, %10\n\tds_read_b64 %5, %10 offset:256\n\t"
                "ds_read_b64 %6, %11\n\tds_read_b64 %7, %11 offset:256\n\ts_waitcnt lgkmcnt(0)"
                : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),
                  "=&v"(v[7])
                : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3])
                : "memory");
#pragma unroll
            for (int j = 0; j < 4; j++) s[j] = xor3(s[j], v[2 * j].x ^ v[2 * j].y, v[2 * j + 1].x ^ v[2 * j + 1].y);
        } else {
            uint32_t v[16];
            asm volatile(
                "ds_read_b32 %0, %16\n\tds_read_b32 %1, %16 offset:128\n\tds_read_b32 %2, %16 offset:256\n\t"
                "ds_read_b32 %3, %16 offset:384\n\t"
                "ds_read_b32 %4, %17\n\tds_read_b32 %5, %17 offset:128\n\tds_read_b32 %6, %17 offset:256\n\t"
                "ds_read_b32 %7, %17 offset:384\n\t"
                "ds_read_b32 %8, %18\n\tds_read_b32 %9, %18 offset:128\n\tds_read_b32 %10, %18 offset:256\n\t"
                "ds_read_b32 %11, %18 offset:384\n\t"
                "ds_read_b32 %12, %19\n\tds_read_b32 %13, %19 offset:128\n\tds_read_b32 %14, %19 offset:256\n\t"
                "ds_read_b32 %15, %19 offset:384\n\ts_waitcnt lgkmcnt(0)"
                : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),
                  "=&v"(v[7]), "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11]), "=&v"(v[12]), "=&v"(v[13]),
                  "=&v"(v[14]), "=&v"(v[15])
                : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3])
                : "memory");
#pragma unroll
            for (int j = 0; j < 4; j++) s[j] = xor3(s[j], xor3(v[4 * j], v[4 * j + 1], v[4 * j + 2]), v[4 * j + 3]);
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] ^ s[1] ^ s[2] ^ s[3];
    if (threadIdx.x == 0) {
        clk[blockIdx.x].t0 = t0;
        clk[blockIdx.x].r0 = r0;
        clk[blockIdx.x].t1 = __builtin_amdgcn_s_memtime();
        clk[blockIdx.x].r1 = __builtin_amdgcn_s_memrealtime();
    }
}

// Cross-lane gathers: per iteration 16 lookups, NB of them ds_bpermute_b32
// from a 256-B table held in one VGPR (lane l holds bytes 4l..4l+3: an S-box
// fits), the rest conflict-free ds_read_b32.  Shows whether bpermute, which
// reads no LDS bank, adds gather throughput beside the ds_read_b32 peak.
template <int NB>
__global__ __launch_bounds__(1024, 1) void k_bperm(uint32_t* out, int iters, Clk* clk) {
    __shared__ uint32_t lds[24576];  // 96 KiB: one workgroup per CU
    for (int i = threadIdx.x; i < 24576; i += blockDim.x) lds[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t lo = (threadIdx.x & 31u) << 2;
    const uint32_t tab = threadIdx.x * 0x01010101u + 0x03020100u;
    uint32_t s[16];
#pragma unroll
    for (int j = 0; j < 16; j++) s[j] = (threadIdx.x * 7919u + j * 104729u) | 1;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int it = 0; it < iters; it++) {
        uint32_t v[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            if (j < NB) {
                v[j] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((s[j] >> (8 * (j & 3))) & 0xFCu), (int)tab);
            } else {
                const uint32_t a = __builtin_amdgcn_perm(s[j], lo, 0x0C0C0400u + ((j & 3) << 8));
                v[j] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + a);
            }
        }
#pragma unroll
        for (int j = 0; j < 16; j++) s[j] ^= v[j];
    }
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) acc ^= s[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) {
        clk[blockIdx.x].t0 = t0;
        clk[blockIdx.x].r0 = r0;
        clk[blockIdx.x].t1 = __builtin_amdgcn_s_memtime();
        clk[blockIdx.x].r1 = __builtin_amdgcn_s_memrealtime();
    }
}

// VALU issue: 8 independent chains x 8 unrolled ops of one kind.
template <int OP>
__global__ __launch_bounds__(1024, 1) void k_valu(uint32_t* out, int iters, Clk* clk) {
    __shared__ uint32_t pin[24576];  // 96 KiB: one workgroup per CU
    if (iters < 0) pin[threadIdx.x] = 1;
    uint32_t x[8];
#pragma unroll
    for (int j = 0; j < 8; j++) x[j] = threadIdx.x * 31u + j;
    const uint32_t y = blockIdx.x * 3u + 1, z = threadIdx.x ^ 0x5555u;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (OP == 0) x[j] = __builtin_amdgcn_perm(x[j], z, 0x0C0C0500u + u);
                if (OP == 1) x[j] = xor3(x[j], y, z + u);
                if (OP == 2) x[j] = __builtin_amdgcn_alignbit(x[j], x[(j + 1) & 7], 8 + u);
            }
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) acc ^= x[j];
    if (iters < 0) acc ^= pin[threadIdx.x ^ 1];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) {
        clk[blockIdx.x].t0 = t0;
        clk[blockIdx.x].r0 = r0;
        clk[blockIdx.x].t1 = __builtin_amdgcn_s_memtime();
        clk[blockIdx.x].r1 = __builtin_amdgcn_s_memrealtime();
    }
}

static const uint32_t* g_tab = nullptr;

template <typename... A>
static void launch(void (*kernel)(uint32_t*, int, Clk*, A...), int grid, int threads, uint32_t* d_out, int iters,
                   Clk* d_clk) {
    if constexpr (sizeof...(A) == 0) hipLaunchKernelGGL(kernel, dim3(grid), dim3(threads), 0, 0, d_out, iters, d_clk);
    else hipLaunchKernelGGL(kernel, dim3(grid), dim3(threads), 0, 0, d_out, iters, d_clk, g_tab);
}

template <typename K>
static void run(const char* name, K kernel, int threads, int iters, double ops_per_thread_iter, const char* unit,
                int cus, uint32_t* d_out, Clk* d_clk) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int grid = cus;
    launch(kernel, grid, threads, d_out, iters / 10, d_clk);  // warm
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    launch(kernel, grid, threads, d_out, iters, d_clk);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    Clk* h = (Clk*)malloc(sizeof(Clk) * grid);
    CHECK(hipMemcpy(h, d_clk, sizeof(Clk) * grid, hipMemcpyDeviceToHost));
    double cyc = 0, real = 0;
    for (int i = 0; i < grid; i++) {
        cyc += (double)(h[i].t1 - h[i].t0);
        real += (double)(h[i].r1 - h[i].r0);
    }
    free(h);
    // Clock from wave 0's s_memtime / s_memrealtime; the rate uses the event
    // time of the whole grid (wave 0 alone finishes early: age priority).
    const double ghz = cyc / real * 0.1;  // s_memrealtime ticks at 100 MHz
    const double total = ops_per_thread_iter * threads * (double)iters;  // per WG (= per CU)
    const double per_clk = total / (ms * 1e-3 * ghz * 1e9);
    printf("{\"test\": \"%s\", \"ms\": %.3f, \"clock_ghz\": %.3f, \"per_cu_per_clk\": %.3f, \"unit\": \"%s\", "
           "\"waves_per_cu\": %d}\n",
           name, ms, ghz, per_clk, unit, threads / 64);
    fflush(stdout);
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t* d_out;
    Clk* d_clk;
    CHECK(hipMalloc(&d_out, (size_t)cus * 1024 * 4));
    CHECK(hipMalloc(&d_clk, (size_t)cus * sizeof(Clk)));
    const int it = 20000;
    uint32_t* d_tab;
    CHECK(hipMalloc(&d_tab, 1024));
    CHECK(hipMemset(d_tab, 0x5a, 1024));
    g_tab = d_tab;
    if (getenv("MB_ONLY_VMIX")) {
        // rates in LDS lookups per clk per CU (the VMEM gathers ride along)
        run("vmix_lds16", k_vmix<0, 0>, 1024, it, 16, "lds lookups", cus, d_out, d_clk);
        run("vmix_lds16_vmem2_d0", k_vmix<2, 0>, 1024, it, 16, "lds lookups", cus, d_out, d_clk);
        run("vmix_lds16_vmem2_d1", k_vmix<2, 1>, 1024, it, 16, "lds lookups", cus, d_out, d_clk);
        run("vmix_lds16_vmem4_d0", k_vmix<4, 0>, 1024, it, 16, "lds lookups", cus, d_out, d_clk);
        run("vmix_lds16_vmem4_d1", k_vmix<4, 1>, 1024, it, 16, "lds lookups", cus, d_out, d_clk);
        run("vmix_lds16_vmem8_d1", k_vmix<8, 1>, 1024, it, 16, "lds lookups", cus, d_out, d_clk);
        run("vmix_lds16_vmem16_d1", k_vmix<16, 1>, 1024, it, 16, "lds lookups", cus, d_out, d_clk);
        return 0;
    }
    if (getenv("MB_ONLY_BPERM")) {
        run("bperm0_lds16", k_bperm<0>, 1024, it, 16, "lookups", cus, d_out, d_clk);
        run("bperm4_lds12", k_bperm<4>, 1024, it, 16, "lookups", cus, d_out, d_clk);
        run("bperm8_lds8", k_bperm<8>, 1024, it, 16, "lookups", cus, d_out, d_clk);
        run("bperm16", k_bperm<16>, 1024, it, 16, "lookups", cus, d_out, d_clk);
        return 0;
    }
    // lane-ops per clk per CU (64 lanes x wave-instructions)
    run("valu_perm", k_valu<0>, 1024, it, 64, "lane-ops", cus, d_out, d_clk);
    run("valu_bitop3", k_valu<1>, 1024, it, 64, "lane-ops", cus, d_out, d_clk);
    run("valu_alignbit", k_valu<2>, 1024, it, 64, "lane-ops", cus, d_out, d_clk);
    run("valu_perm_4waves", k_valu<0>, 256, it, 64, "lane-ops", cus, d_out, d_clk);
    // lookups per clk per CU
    run("lds_gather_x0", k_lds<0>, 1024, it, 16, "lookups", cus, d_out, d_clk);
    run("lds_gather_x1", k_lds<1>, 1024, it, 16, "lookups", cus, d_out, d_clk);
    run("lds_gather_x2", k_lds<2>, 1024, it, 16, "lookups", cus, d_out, d_clk);
    run("lds_gather_x3", k_lds<3>, 1024, it, 16, "lookups", cus, d_out, d_clk);
    run("lds_gather_x0_8waves", k_lds<0>, 512, it, 16, "lookups", cus, d_out, d_clk);
    run("lds_gather_x0_4waves", k_lds<0>, 256, it, 16, "lookups", cus, d_out, d_clk);
    run("lds_peak_b32", k_ldspeak<false>, 1024, it, 16, "ds_read_b32 lanes", cus, d_out, d_clk);
    run("lds_peak_b64", k_ldspeak<true>, 1024, it, 8, "ds_read_b64 lanes", cus, d_out, d_clk);
    run("lds_peak_b32_8w", k_ldspeak<false>, 512, it, 16, "ds_read_b32 lanes", cus, d_out, d_clk);
    run("mix_vmem0", k_mix<0>, 1024, it, 16, "lookups", cus, d_out, d_clk);
    run("mix_vmem2", k_mix<2>, 1024, it, 16, "lookups", cus, d_out, d_clk);
    run("mix_vmem4", k_mix<4>, 1024, it, 16, "lookups", cus, d_out, d_clk);
    run("mix_vmem6", k_mix<6>, 1024, it, 16, "lookups", cus, d_out, d_clk);
    run("mix_vmem16", k_mix<16>, 1024, it / 4, 16, "lookups", cus, d_out, d_clk);
    run("bperm0_lds16", k_bperm<0>, 1024, it, 16, "lookups", cus, d_out, d_clk);
    run("bperm4_lds12", k_bperm<4>, 1024, it, 16, "lookups", cus, d_out, d_clk);
    run("bperm8_lds8", k_bperm<8>, 1024, it, 16, "lookups", cus, d_out, d_clk);
    run("bperm16", k_bperm<16>, 1024, it, 16, "lookups", cus, d_out, d_clk);
    CHECK(hipFree(d_tab));
    CHECK(hipFree(d_out));
    CHECK(hipFree(d_clk));
    return 0;
}
