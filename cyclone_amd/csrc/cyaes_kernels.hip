// cyaes_kernels.hip -- gfx950 (CDNA4) kernels for cyCrypt AES-128-CBC.
//
// Reference: thejinchao/cyclone source/cyCrypt/crypt/cyr_rijndael.cpp
//   encrypt :588-609 (CBC chain) + _encryptBlock :638-705
//   decrypt :612-635 (CBC chain) + _decryptBlock :708-774
//
// Design:
//  * Cipher state is the block loaded as four little-endian dwords, i.e. the
//    byte-swap of the reference's big-endian words (cyr_rijndael.cpp:641-656).
//    Tables and round keys are byte-swapped once on the host, so no swaps run
//    on the device.
//  * T-tables live in LDS as 256 rows x 256 B: row x holds A[x] replicated in
//    32 slots and B[x] in the next 32.  A lookup address is (x << 8) |
//    (lane&31)*4, and lane l always hits bank l%32: the gathers are
//    bank-conflict-free.  The address is one v_perm_b32 (half-rate on gfx950),
//    or for byte 1, already on the row bits, one full-rate v_bitop3_b32.  A
//    second 64 KiB region is selected through byte 2 of the lane-offset
//    register.  Both directions keep all four T-tables (T1|T3, T2|T4): a
//    column is  xor3(T1[b0], T2[b1], xor3(T3[b2], T4[b3], k))  (tcol).
//    Decrypt fills the whole 160 KiB: TL5|TL7, TL6|TL8 and a 32 KiB Si image
//    with 128-B rows.  The last round's S-box bytes come from T-table bytes
//    (encrypt) or the Si x 0x01010101 image (decrypt), merged with bitop3.
//  * Round keys are wave-uniform and live in SGPRs (s_load from the key table;
//    a per-payload key index is handled by a waterfall over the distinct keys
//    present in a wave, normally one).
//  * Encrypt (serial CBC): one lane = one payload chain, 8 blocks (128 B, one
//    full line per lane) loaded per step, the next step's 8 loads in flight
//    during this step's rounds through one load path (a partial last step
//    loads the payload's last 8 blocks), so a step never waits for the
//    previous step's stores (k_encrypt).  Batches with too few chains to fill
//    the chip (uniform or ragged) use four lanes per chain, one state word
//    each, exchanging lookups by DPP quad_perm (k_encrypt_quad).
//  * Decrypt (block-parallel): one lane = one 16-B block, four rows decrypted
//    together, each wave-instruction loads 1 KiB contiguous; the previous
//    ciphertext block comes from the neighbour lane (DPP wave_shr:1), the
//    wave's chain across rows and steps through readlane 63 (k_decrypt_flat;
//    sessions that are whole steps pick their schedule per step).  Ragged
//    batches pack groups of up to 64 payloads into the rows (k_decrypt_ragged).
//  * Waves of a workgroup are kept level by progress-feedback priority
//    (prio_feedback), so none runs a starved tail.
//
// Translation units (r03), each compiled with the LLVM machine scheduler that
// measured best for its kernels (Makefile SCHED_*, profiles/r03/ab_sched.txt):
//   cyaes_kernels.hip      (this file, default scheduler): k_encrypt_quad,
//                          key expansion, workload utilities, the debug
//                          readers that sum every TU's records;
//   cyaes_enc_kernels.hip  (iterative ILP): k_encrypt, k_encrypt_lines;
//   cyaes_dec_kernels.hip  (max ILP): k_decrypt_flat, k_dec_prepass;
//   cyaes_duplex_kernels.hip (iterative ILP): k_duplex;
//   cyaes_ragged_kernels.hip (iterative ILP, r05): k_decrypt_ragged.
// Shared device code (access layer, table lookups, rounds, key schedules,
// priority feedback) is in cyaes_device.h.
//
// Build variants (Makefile): CYAES_CLOCK_PROBE (bench.py's in-kernel clock)
// and CYAES_BOUNDS_CHECK (every global access checked against the extent the
// batch contract gives it; misses are counted, never faulted).  The rejected
// A/B variants of rounds 1-3 are recorded in profiles/r0{1,2,3}/ab_*.txt.
#define CYAES_TU 0
#include "cyaes_device.h"

#include <algorithm>

namespace cyaes {
namespace {

// ---- CBC encrypt, latency-bound batches: four lanes per payload chain ------
// A lane per chain (k_encrypt) fills the chip only with >= 16 waves of chains
// per CU; below that each wave is a serial chain of ~40 dependent VALU/LDS
// instructions per round.  Here a quad of lanes shares one chain: lane q owns
// state word q.  Per round it looks up the four bytes of its own word (T1..T4
// as tcol) and the quad exchanges them with DPP quad_perm: column j =
// T1[b0(s_j)] ^ T2[b1(s_j+1)] ^ T3[b2(s_j+2)] ^ T4[b3(s_j+3)] ^ k_j
// (cyr_rijndael.cpp:659-682), so a round is ~12 instructions on the chain's
// critical path instead of ~40.  Round-key words are per lane (word q of each
// round key) in VGPRs, so per-payload keys need no waterfall.
constexpr uint32_t kQuadFrom1 = 0x39;  // quad_perm [1,2,3,0]: lane j reads lane j+1
constexpr uint32_t kQuadFrom2 = 0x4E;  // [2,3,0,1]
constexpr uint32_t kQuadFrom3 = 0x93;  // [3,0,1,2]
template <uint32_t CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}

// One AES block on a quad: s = word q of (plaintext ^ chain ^ k0) in, word q of the ciphertext out.
__device__ __forceinline__ uint32_t enc_block_quad(const char* lds, uint32_t lo, const uint32_t (&k)[11], uint32_t s) {
#pragma unroll
    for (int r = 1; r < 10; r++) {
        const uint32_t a0 = ld(lds, addr(s, lo, kSel0));                    // T1[b0(s_q)] -> column q
        const uint32_t a1 = ld(lds, addr1(s, lo));                          // T2[b1(s_q)] -> column q-1
        const uint32_t a2 = ld(lds + kHalfB, addr(s, lo, kSel2));           // T3[b2(s_q)] -> column q-2
        const uint32_t a3 = ld(lds + kHalfB, addr(s, lo, region1(kSel3)));  // T4[b3(s_q)] -> column q-3
        s = xor3(a0, qperm<kQuadFrom1>(a1), xor3(qperm<kQuadFrom2>(a2), qperm<kQuadFrom3>(a3), k[r]));
    }
    const uint32_t l0 = ld(lds + kHalfB, addr(s, lo, kSel0));   // S in byte 0 (TL3)
    const uint32_t l1 = ld(lds + kHalfB, addr1(s, lo));         // byte 1 (TL4)
    const uint32_t l2 = ld(lds, addr(s, lo, kSel2));            // byte 2 (TL1)
    const uint32_t l3 = ld(lds, addr(s, lo, region1(kSel3)));   // byte 3 (TL2)
    return merge4(l0, qperm<kQuadFrom1>(l1), qperm<kQuadFrom2>(l2), qperm<kQuadFrom3>(l3)) ^ k[10];
}

template <bool RAGGED, bool KEYED>
__global__ __launch_bounds__(kEncThreads, 1) void k_encrypt_quad(EncArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_words[kEncLdsWords];
    fill_region(lds_words, a.tables, a.tables + 512, blockDim.x);              // TL1 | TL3
    fill_region(lds_words + 16384, a.tables + 256, a.tables + 768, blockDim.x);  // TL2 | TL4
    __shared__ uint32_t lead;  // prio_feedback
    if (threadIdx.x == 0) lead = 0;
    uint32_t prog = 0;
    __syncthreads();
    CLOCK_PROBE(0);
    const char* lds = reinterpret_cast<const char*>(lds_words);
    const uint32_t q = threadIdx.x & 3u;
    const uint32_t lo = ((threadIdx.x & 31u) << 2) | 0x10000u;
    const uint64_t nquads = (uint64_t)gridDim.x * (blockDim.x / 4);
    const Ext iv_in_e = iv_ext(a.iv_in, a.npayloads), iv_out_e = iv_ext(a.iv_out, a.npayloads);
    const Ext key_e = key_ext(a.keys);
    // Every lane of a wave runs the loop the same number of times (the bound
    // is per wave), so a quad never waits in a branch its partners skipped.
    const uint64_t wq0 = (uint64_t)blockIdx.x * (blockDim.x / 4) + __builtin_amdgcn_readfirstlane(threadIdx.x / 4 & ~15u);
    for (uint64_t wq = wq0; wq < a.npayloads; wq += nquads) {
        const uint64_t p = wq + (threadIdx.x / 4 & 15u);
        if (p >= a.npayloads) continue;
        uint64_t off;
        uint32_t nb;
        if (RAGGED && a.stride) {  // strided batch
            off = a.off0 + p * a.stride;
            nb = a.payload_bytes >> 4;
        } else if (RAGGED) {
            off = LD8(a.offsets + p, ext(a.offsets, 8 * a.npayloads));
            nb = LD4(a.nbytes + p, ext(a.nbytes, 4 * a.npayloads)) >> 4;
        } else {
            off = p * (uint64_t)a.payload_bytes;
            nb = a.payload_bytes >> 4;
        }
        const uint32_t kid = KEYED ? key_index(a.keys, p, a.npayloads, true, a.status) : 0u;
        uint32_t k[11];
        const uint32_t* sched = a.keys.table + (uint64_t)kid * kSchedWords + q;
#pragma unroll
        for (int r = 0; r < 11; r++) k[r] = LD4(sched + 4 * r, key_e);
        uint32_t c = a.iv_in ? LD4(a.iv_in + 16 * p + 4 * q, iv_in_e) : (kIv0 + 0x04040404u * q);
        const Ext se = ext(a.in + off, 16ull * nb), de = ext(a.out + off, 16ull * nb);  // this payload's bytes
        const uint8_t* src = a.in + off + 4 * q;  // word q of block i at src + 16 i
        uint8_t* dst = a.out + off + 4 * q;
        auto ldw = [&](uint32_t i) { return LD4(src + 16ull * i, se); };
        uint32_t i = 0;
        uint32_t b[8];
        if (nb >= 8) {
#pragma unroll
            for (int j = 0; j < 8; j++) b[j] = ldw(j);
        }
        for (; i + 8 <= nb; i += 8) {
            uint32_t bn[8];  // next chunk's loads in flight during this chunk's rounds
            const bool more = i + 16 <= nb;
            if (more) {
#pragma unroll
                for (int j = 0; j < 8; j++) bn[j] = ldw(i + 8 + j);
            }
            prio_feedback(&lead, ++prog, kEncPrioDiv);
#pragma unroll
            for (int j = 0; j < 8; j++) {
                c = enc_block_quad(lds, lo, k, xor3(c, b[j], k[0]));
                b[j] = c;
            }
#pragma unroll
            for (int j = 0; j < 8; j++) ST4(dst + 16ull * (i + j), de, b[j]);
            if (more) {
#pragma unroll
                for (int j = 0; j < 8; j++) b[j] = bn[j];
            }
        }
        for (; i < nb; i++) {
            c = enc_block_quad(lds, lo, k, xor3(c, ldw(i), k[0]));
            ST4(dst + 16ull * i, de, c);
        }
        if (a.iv_out) ST4(a.iv_out + 16 * p + 4 * q, iv_out_e, c);
    }
}

// ---- key schedule (Rijndael::Rijndael, cyr_rijndael.cpp:507-572) ----------
__device__ __forceinline__ uint32_t xt(uint32_t a) { return ((a << 1) ^ ((a & 0x80u) ? 0x1bu : 0u)) & 0xffu; }
__device__ __forceinline__ uint32_t gm(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 0; i < 4; i++) {
        if (b & (1u << i)) r ^= a;
        a = xt(a);
    }
    return r;
}

__global__ void k_key_expand(const uint8_t* keys, uint32_t nkeys, const uint8_t* sbox, uint32_t* sched) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nkeys) return;
    uint32_t w[44];  // big-endian words, reference layout m_Ke
    for (int j = 0; j < 4; j++) {
        const uint8_t* k = keys + 16ull * i + 4 * j;
        w[j] = ((uint32_t)k[0] << 24) | ((uint32_t)k[1] << 16) | ((uint32_t)k[2] << 8) | k[3];
    }
    uint32_t rcon = 1;
    for (int j = 4; j < 44; j++) {
        uint32_t t = w[j - 1];
        if ((j & 3) == 0) {
            t = ((uint32_t)sbox[(t >> 16) & 0xff] << 24) ^ ((uint32_t)sbox[(t >> 8) & 0xff] << 16) ^
                ((uint32_t)sbox[t & 0xff] << 8) ^ (uint32_t)sbox[t >> 24] ^ (rcon << 24);
            rcon = xt(rcon);
        }
        w[j] = w[j - 4] ^ t;
    }
    // Device layout (cyaes_internal.h): LE words.
    uint32_t* s = sched + (uint64_t)i * kSchedWords;
    for (int j = 0; j < 44; j++) s[j] = __builtin_bswap32(w[j]);
    for (int r = 0; r <= 10; r++) {
        for (int c = 0; c < 4; c++) {
            uint32_t t = w[4 * (10 - r) + c];
            if (r >= 1 && r <= 9) {  // InvMixColumn (cyr_rijndael.cpp:563-571)
                const uint32_t b0 = t >> 24, b1 = (t >> 16) & 0xff, b2 = (t >> 8) & 0xff, b3 = t & 0xff;
                t = ((gm(b0, 14) ^ gm(b1, 11) ^ gm(b2, 13) ^ gm(b3, 9)) << 24) |
                    ((gm(b0, 9) ^ gm(b1, 14) ^ gm(b2, 11) ^ gm(b3, 13)) << 16) |
                    ((gm(b0, 13) ^ gm(b1, 9) ^ gm(b2, 14) ^ gm(b3, 11)) << 8) |
                    (gm(b0, 11) ^ gm(b1, 13) ^ gm(b2, 9) ^ gm(b3, 14));
            }
            s[44 + 4 * r + c] = __builtin_bswap32(t);
        }
    }
}

// ---- workload utilities --------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_fill_synthetic(uint64_t* buf, uint64_t p0, uint64_t npayloads, uint32_t words_pp, uint64_t seed) {
    const uint64_t total = npayloads * words_pp;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
        const uint64_t p = t / words_pp;
        const uint64_t w = t - p * words_pp;
        buf[t] = splitmix64(seed + ((p0 + p) << 20) + w);
    }
}

__global__ void k_digest(const uint64_t* buf, uint64_t nwords, unsigned long long* out2) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t x = 0, s = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += stride) {
        const uint64_t h = splitmix64(buf[i] ^ splitmix64(i));
        x ^= h;
        s += h;
    }
    for (int o = 32; o > 0; o >>= 1) {
        x ^= __shfl_xor(x, o);
        s += __shfl_xor(s, o);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicXor(&out2[0], (unsigned long long)x);
        atomicAdd(&out2[1], (unsigned long long)s);
    }
}

}  // namespace

hipError_t launch_encrypt_quad(const EncArgs& a, int grid, int threads, hipStream_t stream) {
    const bool keyed = a.keys.key_idx != nullptr || a.keys.ppk.d != 0;
    const bool ragged = a.offsets != nullptr || a.stride != 0;
    const dim3 g(grid), b(threads);
    if (ragged && keyed) hipLaunchKernelGGL((k_encrypt_quad<true, true>), g, b, 0, stream, a);
    else if (ragged) hipLaunchKernelGGL((k_encrypt_quad<true, false>), g, b, 0, stream, a);
    else if (keyed) hipLaunchKernelGGL((k_encrypt_quad<false, true>), g, b, 0, stream, a);
    else hipLaunchKernelGGL((k_encrypt_quad<false, false>), g, b, 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_key_expand(const uint8_t* d_keys, uint32_t nkeys, const uint8_t* d_sbox, uint32_t* d_sched,
                             hipStream_t stream) {
    const int threads = 64;
    const int grid = (int)((nkeys + threads - 1) / threads);
    hipLaunchKernelGGL(k_key_expand, dim3(grid), dim3(threads), 0, stream, d_keys, nkeys, d_sbox, d_sched);
    return hipGetLastError();
}

// The ragged lists of a strided batch (cyaes_gpu_*_strided fallbacks):
// offsets[p] = first + p * stride, nbytes[p] = payload_bytes.
__global__ void k_strided_lists(uint64_t* offsets, uint32_t* nbytes, uint64_t first, uint64_t stride, uint64_t n,
                                uint32_t payload_bytes) {
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x) {
        offsets[p] = first + p * stride;
        nbytes[p] = payload_bytes;
    }
}

hipError_t launch_strided_lists(uint64_t* offsets, uint32_t* nbytes, uint64_t first, uint64_t stride, uint64_t n,
                                uint32_t payload_bytes, hipStream_t stream) {
    const int threads = 256;
    const uint64_t want = (n + threads - 1) / threads;
    const int grid = (int)(want < 4096 ? (want ? want : 1) : 4096);
    hipLaunchKernelGGL(k_strided_lists, dim3(grid), dim3(threads), 0, stream, offsets, nbytes, first, stride, n,
                       payload_bytes);
    return hipGetLastError();
}

hipError_t launch_fill_synthetic(uint8_t* buf, uint64_t p0, uint64_t npayloads, uint32_t payload_bytes, uint64_t seed,
                                 hipStream_t stream) {
    const int threads = 256;
    const uint64_t total = npayloads * (payload_bytes / 8);
    const uint64_t want = (total + threads - 1) / threads;
    const int grid = (int)(want < 65536 ? (want ? want : 1) : 65536);
    hipLaunchKernelGGL(k_fill_synthetic, dim3(grid), dim3(threads), 0, stream, reinterpret_cast<uint64_t*>(buf), p0,
                       npayloads, payload_bytes / 8, seed);
    return hipGetLastError();
}

hipError_t launch_digest(const uint8_t* buf, uint64_t nwords, unsigned long long* out2, hipStream_t stream) {
    const int threads = 256;
    const uint64_t want = (nwords + threads - 1) / threads;
    const int grid = (int)(want < 8192 ? (want ? want : 1) : 8192);
    hipLaunchKernelGGL(k_digest, dim3(grid), dim3(threads), 0, stream, reinterpret_cast<const uint64_t*>(buf), nwords,
                       out2);
    return hipGetLastError();
}

}  // namespace cyaes

#if CYAES_CLOCK_PROBE
// Reads and clears the probe sums of every kernel TU: out[8] = (enc, dec) x
// {cycles, ticks, waves, max ticks}.
extern "C" int cyaes_debug_probe(unsigned long long* out) {
    unsigned long long part[5][8];
    if (cyaes::read_probe_local(part[0]) || cyaes::probe_read_enc(part[1]) || cyaes::probe_read_dec(part[2]) ||
        cyaes::probe_read_dup(part[3]) || cyaes::probe_read_rag(part[4]))
        return -1;
    for (int i = 0; i < 8; i++) {
        out[i] = 0;
        for (int t = 0; t < 5; t++) out[i] = (i % 4 == 3) ? std::max(out[i], part[t][i]) : out[i] + part[t][i];
    }
    return 0;
}

// Per-wave timeline of the last launch of a kind (0 encrypt, 1 decrypt) in one
// kernel translation unit (0: this one -- quad encrypt; 1: the lane encrypt;
// 2: the flat decrypt; 3: the duplex kernel, kind 0 its encrypt phase and
// kind 1 its decrypt phase; 4: the ragged decrypt): kTimelineWaves x 2 uint4
// (cyaes_device.h), read and cleared.  tools/timeline.py.
extern "C" int cyaes_debug_timeline(int tu, int kind, void* out) {
    if (kind < 0 || kind > 1) return -1;
    uint4* o = static_cast<uint4*>(out);
    if (tu == 0) return cyaes::read_timeline_local(kind, o);
    if (tu == 1) return cyaes::timeline_read_enc(kind, o);
    if (tu == 2) return cyaes::timeline_read_dec(kind, o);
    if (tu == 3) return cyaes::timeline_read_dup(kind, o);
    if (tu == 4) return cyaes::timeline_read_rag(kind, o);
    return -1;
}
#endif

#if CYAES_BOUNDS_CHECK
// Reads and clears the bounds records of every kernel TU: out[4] = misses, the
// first miss's source position (TU * 10000 + line: 0 cyaes_kernels.hip, 1
// cyaes_enc_kernels.hip, 2 cyaes_dec_kernels.hip, 3 cyaes_duplex_kernels.hip,
// 4 cyaes_ragged_kernels.hip),
// its offset from the extent's start, the extent's size; then up to 8
// (position, misses) pairs in out[4..20).
extern "C" int cyaes_debug_bounds(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    static unsigned long long rec[5][4];
    static unsigned int lines[5][cyaes::kBoundsLines];
    if (cyaes::read_bounds_local(rec[0], lines[0]) || cyaes::bounds_read_enc(rec[1], lines[1]) ||
        cyaes::bounds_read_dec(rec[2], lines[2]) || cyaes::bounds_read_dup(rec[3], lines[3]) ||
        cyaes::bounds_read_rag(rec[4], lines[4]))
        return -1;
    for (int i = 0; i < 20; i++) out[i] = 0;
    for (int t = 0; t < 5; t++) {
        if (rec[t][0] && !out[0]) out[1] = 10000ull * t + rec[t][1], out[2] = rec[t][2], out[3] = rec[t][3];
        out[0] += rec[t][0];
    }
    for (uint32_t t = 0, k = 4; t < 5; t++)
        for (uint32_t l = 0; l < cyaes::kBoundsLines && k < 20; l++)
            if (lines[t][l]) out[k++] = 10000ull * t + l, out[k++] = lines[t][l];
    return 0;
}
#endif
