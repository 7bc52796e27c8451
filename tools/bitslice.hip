// tools/bitslice.hip -- measurement prototype: bitsliced AES-128 CBC decrypt on
// gfx950, no LDS, against the product's T-table decrypt (k_decrypt_flat via
// libcyaes.so) in the same process.  Answers VERDICT r1 "next round" item 2:
// how many full-rate VALU ops per block, and how many clocks per block per CU,
// does a lookup-free AES decrypt cost on this chip (the T-table path is bound
// at ~5.3 clk/block/CU by LDS gathers)?
//
// What it re-expresses: _decryptBlock (cyr_rijndael.cpp:708-774) and the CBC
// chain of decrypt (:612-635) with iv = nullptr per payload (relay semantics).
//
// Layout (tools/gen_bitslice.py, tools/bitslice_gen.h): a wave takes 512
// consecutive blocks; quad q (lanes 4q..4q+3) holds blocks base + 16 j + q,
// j = 0..31; lane c of the quad loads word c of its 32 blocks (one coalesced
// 256-B global_load_dword per j), transposes the 32x32 bit matrix, and holds
// state column c as 32 registers (register p = 8 * row + bit, bit j = block j).
// InvShiftRows = DPP quad_perm between the quad's lanes; InvSubBytes /
// InvMixColumns / AddRoundKey are the generated v_bitop3_b32 networks; the
// round keys are per-lane 0/~0 masks loaded from a 5.6 KiB table (L1/L2).
//
// usage: bitslice [payloads (64 KiB each), default 262144] [reps, default 5] [waves/WG 16|8]
// build: make -C <repo> build/bitslice
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../include/cyaes.h"
#include "bitslice_gen.h"

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

namespace {

// ---- 32x32 bit transpose, MSB-first convention: out[i] bit (31-k) = in[k] bit (31-i)
template <int J>
__device__ __forceinline__ void tstage(uint32_t (&w)[32]) {
    constexpr uint32_t M = J == 16 ? 0x0000FFFFu : J == 8 ? 0x00FF00FFu : J == 4 ? 0x0F0F0F0Fu
                         : J == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
    for (int k = 0; k < 32; k = (k + J + 1) & ~J) {
        const uint32_t a = w[k], b = w[k + J];
        // a' = (a & ~M) | ((b >> J) & M);  b' = (b & ~(M << J)) | ((a << J) & (M << J)):
        // S2 ? S1 : S0 = 0xD8 (S0 = 0xF0, S1 = 0xCC, S2 = 0xAA)
        w[k] = __builtin_amdgcn_bitop3_b32(a, b >> J, M, 0xD8);
        w[k + J] = __builtin_amdgcn_bitop3_b32(b, a << J, M << J, 0xD8);
    }
}
__device__ __forceinline__ void transpose32(uint32_t (&w)[32]) {
    tstage<16>(w);
    tstage<8>(w);
    tstage<4>(w);
    tstage<2>(w);
    tstage<1>(w);
}

template <uint32_t CTRL>
__device__ __forceinline__ uint32_t qp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
// InvShiftRows: lane c takes row r from lane c - r (mod 4).
__device__ __forceinline__ void inv_shift_rows(uint32_t (&v)[32]) {
#pragma unroll
    for (int b = 0; b < 8; b++) {
        v[8 + b] = qp<0x93>(v[8 + b]);   // [3,0,1,2]: from lane c-1
        v[16 + b] = qp<0x4E>(v[16 + b]); // [2,3,0,1]: from lane c-2
        v[24 + b] = qp<0x39>(v[24 + b]); // [1,2,3,0]: from lane c-3
    }
}

__device__ unsigned long long g_probe[4];  // cycles, ticks, waves, max ticks

template <int WAVES>
__global__ __launch_bounds__(64 * WAVES, 1) void k_bs_decrypt(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                           uint64_t nblocks, uint32_t bpp,
                                                           const uint32_t* __restrict__ masks) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t lane = threadIdx.x & 63u, q = lane >> 2, c = lane & 3u;
    const uint64_t nwaves = (uint64_t)gridDim.x * WAVES;
    const uint64_t wave = (uint64_t)blockIdx.x * WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t ngroups = nblocks / 512;  // (the harness sizes batches in whole 512-block groups)
    for (uint64_t grp = wave; grp < ngroups; grp += nwaves) {
        const uint64_t base = grp * 512;
        const uint32_t* src = in + (base + q) * 4 + c;  // block base + 16 j + q, word c: src[64 j]
        uint32_t* dst = out + (base + q) * 4 + c;
        uint32_t v[32];
#pragma unroll
        for (int j = 0; j < 32; j++) v[j] = src[64 * j];
        transpose32(v);
        uint32_t s[32];
#pragma unroll
        for (int p = 0; p < 32; p++) s[p] = v[31 - p];
        const uint32_t* mc = masks + 32 * c;  // this lane's column; round r at + 128 r
        bs::init(s, mc);
#pragma unroll 1
        for (int r = 1; r < 10; r++) {
            inv_shift_rows(s);
            bs::middle(s, mc + 128 * r);
        }
        inv_shift_rows(s);
        bs::last(s, mc + 128 * 10);
#pragma unroll
        for (int p = 0; p < 32; p++) v[31 - p] = s[p];
        transpose32(v);
        // CBC: xor the previous ciphertext block (DefaultIV at a payload start)
        // (bpp is a power of two >= 512: only block `base` of the group can start a payload)
        const bool start = (base & (bpp - 1)) == 0;
#pragma unroll
        for (int j = 0; j < 32; j++) {
            const uint32_t iv = 0x03020100u + 0x04040404u * c;
            const uint32_t prev = (j == 0 && q == 0 && start) ? iv : src[64 * j - 4];
            dst[64 * j] = v[j] ^ prev;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        atomicAdd(&g_probe[0], (unsigned long long)(t1 - t0));
        atomicAdd(&g_probe[1], (unsigned long long)(r1 - r0));
        atomicAdd(&g_probe[2], 1ull);
        atomicMax(&g_probe[3], (unsigned long long)(r1 - r0));
    }
}

__global__ void k_count_diff(const uint32_t* a, const uint32_t* b, uint64_t n, unsigned long long* bad) {
    uint64_t local = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        local += a[i] != b[i];
    if (local) atomicAdd(bad, (unsigned long long)local);
}

__global__ void k_fill(uint64_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + i * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

// ---- host: round keys of the equivalent inverse cipher, in bytes ------------
uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }
uint8_t gm(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    for (int i = 0; i < 8; i++, a = xt(a), b >>= 1)
        if (b & 1) r ^= a;
    return r;
}
uint8_t sbox(uint8_t x) {
    uint8_t inv = 0;
    for (int y = 1; y < 256 && x; y++)
        if (gm(x, (uint8_t)y) == 1) inv = (uint8_t)y;
    uint8_t r = 0;
    for (int i = 0; i < 8; i++) {
        const int bit = ((inv >> i) ^ (inv >> ((i + 4) % 8)) ^ (inv >> ((i + 5) % 8)) ^ (inv >> ((i + 6) % 8)) ^
                         (inv >> ((i + 7) % 8))) & 1;
        r |= (uint8_t)(bit << i);
    }
    return r ^ 0x63;
}
// kd[r][16]: kd[0] = w[40..43], kd[1..9] = InvMixColumns(w[4(10-r)..]), kd[10] = w[0..3] (state byte order)
void round_keys(const uint8_t key[16], uint8_t kd[11][16]) {
    uint8_t S[256];
    for (int x = 0; x < 256; x++) S[x] = sbox((uint8_t)x);
    uint8_t w[176];
    memcpy(w, key, 16);
    uint8_t rcon = 1;
    for (int i = 16; i < 176; i += 4) {
        uint8_t t[4] = {w[i - 4], w[i - 3], w[i - 2], w[i - 1]};
        if (i % 16 == 0) {
            const uint8_t t0 = t[0];
            t[0] = S[t[1]] ^ rcon, t[1] = S[t[2]], t[2] = S[t[3]], t[3] = S[t0];
            rcon = xt(rcon);
        }
        for (int k = 0; k < 4; k++) w[i + k] = w[i - 16 + k] ^ t[k];
    }
    for (int r = 0; r <= 10; r++) {
        const uint8_t* k = w + 16 * (10 - r);
        for (int c = 0; c < 4; c++) {
            const uint8_t* a = k + 4 * c;
            if (r == 0 || r == 10) {
                memcpy(&kd[r][4 * c], a, 4);
            } else {
                kd[r][4 * c + 0] = gm(a[0], 14) ^ gm(a[1], 11) ^ gm(a[2], 13) ^ gm(a[3], 9);
                kd[r][4 * c + 1] = gm(a[0], 9) ^ gm(a[1], 14) ^ gm(a[2], 11) ^ gm(a[3], 13);
                kd[r][4 * c + 2] = gm(a[0], 13) ^ gm(a[1], 9) ^ gm(a[2], 14) ^ gm(a[3], 11);
                kd[r][4 * c + 3] = gm(a[0], 11) ^ gm(a[1], 13) ^ gm(a[2], 9) ^ gm(a[3], 14);
            }
        }
    }
}
uint8_t min_apply(uint8_t x) {
    uint8_t r = 0;
    for (int i = 0; i < 8; i++) r |= (uint8_t)((__builtin_popcount(bs::MIN_ROWS[i] & x) & 1) << i);
    return r;
}

template <int W>
float run_bs(const uint32_t* d_in, uint32_t* d_out, uint64_t nblocks, uint32_t bpp, const uint32_t* d_masks, int cus,
             hipStream_t s) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a, s));
    hipLaunchKernelGGL(k_bs_decrypt<W>, dim3(cus * (16 / W)), dim3(64 * W), 0, s, d_in, d_out, nblocks, bpp, d_masks);
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(b, s));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return ms;
}

}  // namespace

int main(int argc, char** argv) {
    const uint64_t npay = argc > 1 ? strtoull(argv[1], nullptr, 10) : 262144;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const int waves = argc > 3 ? atoi(argv[3]) : 16;
    const uint32_t pb = 65536, bpp = pb / 16;
    const uint64_t nblocks = npay * bpp, nbytes = npay * pb;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint8_t key[16];
    for (int i = 0; i < 16; i++) key[i] = (uint8_t)i;
    uint8_t kd[11][16];
    round_keys(key, kd);
    // masks[r][c][p]: p = 8 row + bit
    std::vector<uint32_t> masks(11 * 4 * 32);
    for (int r = 0; r <= 10; r++)
        for (int c = 0; c < 4; c++)
            for (int row = 0; row < 4; row++) {
                const uint8_t kb = kd[r][4 * c + row];
                const uint8_t mb = r == 10 ? kb : (uint8_t)(min_apply(kb) ^ bs::C_IN);
                for (int bit = 0; bit < 8; bit++) masks[(r * 4 + c) * 32 + 8 * row + bit] = ((mb >> bit) & 1) ? ~0u : 0u;
            }
    uint32_t *d_in, *d_ref, *d_out, *d_masks;
    unsigned long long* d_bad;
    CHECK(hipMalloc(&d_in, nbytes));
    CHECK(hipMalloc(&d_ref, nbytes));
    CHECK(hipMalloc(&d_out, nbytes));
    CHECK(hipMalloc(&d_masks, masks.size() * 4));
    CHECK(hipMalloc(&d_bad, 8));
    CHECK(hipMemcpy(d_masks, masks.data(), masks.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(d_in), nbytes / 8, 0xC1C1ull);
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    cyaes_gpu* ctx = nullptr;
    if (cyaes_gpu_create(0, &ctx) || cyaes_gpu_set_keys(ctx, key, 1)) {
        fprintf(stderr, "cyaes context failed\n");
        return 1;
    }
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    std::vector<float> t_ref, t_bs;
    unsigned long long probe[4] = {0, 0, 0, 0}, zero[4] = {0, 0, 0, 0};
    for (int rep = 0; rep <= reps; rep++) {
        CHECK(hipEventRecord(a, s));
        if (cyaes_gpu_decrypt_uniform(ctx, reinterpret_cast<uint8_t*>(d_in), reinterpret_cast<uint8_t*>(d_ref), npay, pb,
                                      nullptr, 0, nullptr, nullptr, s)) {
            fprintf(stderr, "reference decrypt failed\n");
            return 1;
        }
        CHECK(hipEventRecord(b, s));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_probe), zero, sizeof(zero)));
        const float mb = waves == 8 ? run_bs<8>(d_in, d_out, nblocks, bpp, d_masks, cus, s)
                                    : run_bs<16>(d_in, d_out, nblocks, bpp, d_masks, cus, s);
        if (rep == 0) {  // warm-up; check
            CHECK(hipMemset(d_bad, 0, 8));
            hipLaunchKernelGGL(k_count_diff, dim3(8192), dim3(256), 0, s, d_out, d_ref, nbytes / 4, d_bad);
            unsigned long long bad = 0;
            CHECK(hipMemcpy(&bad, d_bad, 8, hipMemcpyDeviceToHost));
            printf("{\"check\": \"bitsliced vs libcyaes k_decrypt_flat\", \"mismatched_words\": %llu, \"words\": %llu}\n",
                   bad, (unsigned long long)(nbytes / 4));
            if (bad) return 2;
            continue;
        }
        unsigned long long pr[4];
        CHECK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_probe), sizeof(pr)));
        for (int i = 0; i < 3; i++) probe[i] += pr[i];
        t_ref.push_back(ms);
        t_bs.push_back(mb);
    }
    std::sort(t_ref.begin(), t_ref.end());
    std::sort(t_bs.begin(), t_bs.end());
    const double ghz = probe[1] ? (double)probe[0] / probe[1] * 0.1 : 0;
    const double med_bs = t_bs[t_bs.size() / 2], med_ref = t_ref[t_ref.size() / 2];
    const double clk_per_block_cu = med_bs * 1e-3 * ghz * 1e9 * cus / (double)nblocks;
    printf("{\"payloads\": %llu, \"payload_bytes\": %u, \"waves_per_cu\": %d, \"bitsliced_ms\": %.3f, "
           "\"ttable_ms\": %.3f, \"ratio\": %.3f, \"bitsliced_clock_ghz\": %.3f, \"bitsliced_clk_per_block_per_cu\": %.3f, "
           "\"bitsliced_GBps\": %.1f, \"ttable_GBps\": %.1f}\n",
           (unsigned long long)npay, pb, waves, med_bs, med_ref, med_bs / med_ref, ghz, clk_per_block_cu,
           2.0 * nbytes / (med_bs * 1e-3) / 1e9, 2.0 * nbytes / (med_ref * 1e-3) / 1e9);
    cyaes_gpu_destroy(ctx);
    return 0;
}
