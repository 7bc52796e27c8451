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
// Build variants (Makefile): CYAES_CLOCK_PROBE (bench.py's in-kernel clock)
// and CYAES_BOUNDS_CHECK (every global access checked against the extent the
// batch contract gives it; misses are counted, never faulted).  The rejected
// A/B variants of rounds 1-2 are recorded in profiles/r0{1,2}/ab_*.txt.
#include "cyaes_internal.h"

#ifndef CYAES_BOUNDS_CHECK
#define CYAES_BOUNDS_CHECK 0
#endif

namespace cyaes {
namespace {

// v_perm_b32 selectors: result = (byte k of u) << 8 | lo.byte0 [| lo.byte2 << 16]
constexpr uint32_t kSel0 = 0x0C0C0400u;
constexpr uint32_t kSel2 = 0x0C0C0600u;
constexpr uint32_t kSel3 = 0x0C0C0700u;
// Region-1 selectors: byte2 = 0x02 picks lo.byte2 (= 1), i.e. + 64 KiB.
constexpr uint32_t region1(uint32_t sel) { return (sel & 0xFF00FFFFu) | 0x00020000u; }
constexpr uint32_t kHalfB = 128;            // byte offset of table B inside a row

// DefaultIV (cyr_rijndael.cpp:503-504) as little-endian dwords.
constexpr uint32_t kIv0 = 0x03020100u, kIv1 = 0x07060504u, kIv2 = 0x0b0a0908u, kIv3 = 0x0f0e0d0cu;

// ---- global accesses --------------------------------------------------------
// Every global load and store of the AES kernels names the extent [lo, hi)
// the batch contract allows it (the payload's bytes, the IV array, the key
// table, ...).  In the CYAES_BOUNDS_CHECK build an access outside it is
// counted in g_bounds (first offender's source line, offset and extent kept)
// and redirected to a sink, so a stray access is reported by name instead of
// faulting the device; cyaes_debug_bounds() reads the record.  In the product
// build the extent is dead code.
struct Ext {
    const uint8_t* lo;
    const uint8_t* hi;
};
__device__ __forceinline__ Ext ext(const void* p, uint64_t bytes) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    return Ext{b, b + bytes};
}

#if CYAES_BOUNDS_CHECK
constexpr uint32_t kBoundsLines = 2048;    // misses per source line of this file
__device__ unsigned long long g_bounds[4];  // misses, first miss's line, its offset from lo, the extent's size
__device__ unsigned int g_bounds_lines[kBoundsLines];
__device__ uint4 g_bounds_sink[64];
template <typename T>
__device__ __forceinline__ T* bchk(T* p, Ext e, uint32_t bytes, uint32_t line) {
    const uint8_t* b = reinterpret_cast<const uint8_t*>(p);
    if (e.lo && b >= e.lo && b + bytes <= e.hi) return p;
    atomicAdd(&g_bounds_lines[line % kBoundsLines], 1u);
    if (atomicAdd(&g_bounds[0], 1ull) == 0) {
        g_bounds[1] = line;
        g_bounds[2] = (unsigned long long)(b - e.lo);
        g_bounds[3] = (unsigned long long)(e.hi - e.lo);
    }
    return reinterpret_cast<T*>(&g_bounds_sink[__lane_id()]);
}
#define AT(p, e, bytes) bchk((p), (e), (bytes), __LINE__)
#else
#define AT(p, e, bytes) ((void)(e), (p))
#endif

// 16-B block at a 4-byte-aligned address (ragged batches: relay packets put
// the payload at packet offset 12).  Still one global_load/store_dwordx4.
struct __attribute__((aligned(4))) Blk4 {
    uint32_t x, y, z, w;
};
#define LD16(p, e) (*AT(reinterpret_cast<const uint4*>(p), (e), 16))
#define ST16(p, e, v) (*AT(reinterpret_cast<uint4*>(p), (e), 16) = (v))
#define LD16U(p, e) blk_in(*AT(reinterpret_cast<const Blk4*>(p), (e), 16))
#define ST16U(p, e, v) (*AT(reinterpret_cast<Blk4*>(p), (e), 16) = blk_out(v))
#define LD4(p, e) (*AT(reinterpret_cast<const uint32_t*>(p), (e), 4))
#define ST4(p, e, v) (*AT(reinterpret_cast<uint32_t*>(p), (e), 4) = (v))
#define LD8(p, e) (*AT(reinterpret_cast<const uint64_t*>(p), (e), 8))
__device__ __forceinline__ uint4 blk_in(Blk4 v) { return make_uint4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ Blk4 blk_out(uint4 v) { return Blk4{v.x, v.y, v.z, v.w}; }

// Block i of a payload at base (extent e): 16-B aligned (U = false) or 4-B aligned (U = true).
template <bool U>
__device__ __forceinline__ uint4 ldb(const uint8_t* base, uint32_t i, Ext e) {
    if (U) return LD16U(base + 16ull * i, e);
    return LD16(base + 16ull * i, e);
}
template <bool U>
__device__ __forceinline__ void stb(uint8_t* base, uint32_t i, uint4 v, Ext e) {
    if (U) ST16U(base + 16ull * i, e, v);
    else ST16(base + 16ull * i, e, v);
}

// Extents of the batch arrays every kernel shares.
__device__ __forceinline__ Ext iv_ext(const uint8_t* iv, uint64_t npayloads) { return ext(iv, 16 * npayloads); }
__device__ __forceinline__ Ext key_ext(const KeySel& ks) { return ext(ks.table, (uint64_t)ks.nkeys * kSchedWords * 4); }

// ---- table lookups ----------------------------------------------------------
__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return __builtin_rotateleft32(x, 8); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// Per bit m ? a : b.  Always v_bitop3_b32 (truth table over S0 = 0xF0,
// S1 = 0xCC, S2 = 0xAA): on gfx950 it issues at the full VALU rate, while
// v_bfi_b32, v_perm_b32, v_and_or_b32 and SDWA forms issue at half of it
// (tools/valurate.hip, profiles/r01/valurate.jsonl).
__device__ __forceinline__ uint32_t sel(uint32_t m, uint32_t a, uint32_t b) {
    return __builtin_amdgcn_bitop3_b32(a, m, b, 0xE2);
}

// Row address of byte k of u: (byte k) << 8 | lane bits (one half-rate v_perm_b32).
__device__ __forceinline__ uint32_t addr(uint32_t u, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(u, lo, sel);
}
// Byte 1 already sits on the row bits: (u & 0xFF00) | lo's other bits, one
// full-rate op.  lo's byte 2 (= 1) makes it a region-1 address, so the tables
// indexed by byte 1 live in region 1.
constexpr uint32_t kRowMask = 0x0000FF00u;
__device__ __forceinline__ uint32_t addr1(uint32_t u, uint32_t lo) { return sel(kRowMask, u, lo); }

__device__ __forceinline__ uint32_t ld(const char* lds, uint32_t a) {
    return *reinterpret_cast<const uint32_t*>(lds + a);
}

// Fill an LDS image: nregions x 64 KiB; region r takes A from tab[512r..] and
// (if has_b[r]) B from tab[512r + 256..].
__device__ __forceinline__ void fill_region(uint32_t* lds, const uint32_t* __restrict__ a,
                                            const uint32_t* __restrict__ b, int threads) {
    uint4* l4 = reinterpret_cast<uint4*>(lds);
    for (int q = threadIdx.x; q < 4096; q += threads) {
        const int half = (q >> 3) & 1;
        if (half && !b) continue;
        const uint32_t v = (half ? b : a)[q >> 4];
        l4[q] = make_uint4(v, v, v, v);
    }
}

__device__ __forceinline__ uint32_t fastdiv(uint32_t n, const Fastdiv& f) {
    if (f.d == 1) return n;  // M = 2^64 does not fit; make_fastdiv leaves 0
    const uint64_t lo = (uint64_t)(uint32_t)f.M * n;
    const uint64_t hi = (f.M >> 32) * n;
    return (uint32_t)((hi + (lo >> 32)) >> 32);
}

// Middle-round column (encrypt TL1..TL4, decrypt TL5..TL8; all four tables
// resident, no rotation).  Image: region 0 = T1 | T3, region 1 = T2 | T4.
__device__ __forceinline__ uint32_t tcol(const char* lds, uint32_t lo, uint32_t x0, uint32_t x1, uint32_t x2,
                                         uint32_t x3, uint32_t k) {
    const uint32_t l0 = ld(lds, addr(x0, lo, kSel0));                   // T1[b0]
    const uint32_t l1 = ld(lds, addr1(x1, lo));                         // T2[b1]
    const uint32_t l2 = ld(lds + kHalfB, addr(x2, lo, kSel2));          // T3[b2]
    const uint32_t l3 = ld(lds + kHalfB, addr(x3, lo, region1(kSel3))); // T4[b3]
    return xor3(l0, l1, xor3(l2, l3, k));
}

// Merge the four last-round bytes (byte j of word j-th lookup).
__device__ __forceinline__ uint32_t merge4(uint32_t l0, uint32_t l1, uint32_t l2, uint32_t l3) {
    return sel(0x0000FFFFu, sel(0x000000FFu, l0, l1), sel(0x00FF0000u, l2, l3));
}

// ---- encryption (_encryptBlock, cyr_rijndael.cpp:638-705) -----------------
// Region 0 rows: A = TL1 (LE bytes 2s,s,s,3s), B = TL3; region 1: A = TL2,
// B = TL4 (TL2/TL3/TL4 = rotl8/16/24 of TL1).  Column j takes b0(u_j),
// b1(u_j+1), b2(u_j+2), b3(u_j+3) (ShiftRows).  Last round: S[x] is byte 0 of
// TL3, byte 1 of TL4, byte 2 of TL1 and byte 3 of TL2.
__device__ __forceinline__ uint32_t enc_last(const char* lds, uint32_t lo, uint32_t x0, uint32_t x1, uint32_t x2,
                                             uint32_t x3) {
    const uint32_t l0 = ld(lds + kHalfB, addr(x0, lo, kSel0));   // TL3
    const uint32_t l1 = ld(lds + kHalfB, addr1(x1, lo));         // TL4
    const uint32_t l2 = ld(lds, addr(x2, lo, kSel2));            // TL1
    const uint32_t l3 = ld(lds, addr(x3, lo, region1(kSel3)));   // TL2
    return merge4(l0, l1, l2, l3);
}

// s = plaintext ^ chain ^ ek[0..3] on entry, ciphertext on exit.
__device__ __forceinline__ void enc_block(const char* lds, uint32_t lo, const uint32_t* __restrict__ ek,
                                          uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3) {
#pragma unroll
    for (int r = 1; r < 10; r++) {
        const uint32_t a0 = tcol(lds, lo, s0, s1, s2, s3, ek[4 * r + 0]);
        const uint32_t a1 = tcol(lds, lo, s1, s2, s3, s0, ek[4 * r + 1]);
        const uint32_t a2 = tcol(lds, lo, s2, s3, s0, s1, ek[4 * r + 2]);
        const uint32_t a3 = tcol(lds, lo, s3, s0, s1, s2, ek[4 * r + 3]);
        s0 = a0; s1 = a1; s2 = a2; s3 = a3;
    }
    const uint32_t o0 = enc_last(lds, lo, s0, s1, s2, s3) ^ ek[40];
    const uint32_t o1 = enc_last(lds, lo, s1, s2, s3, s0) ^ ek[41];
    const uint32_t o2 = enc_last(lds, lo, s2, s3, s0, s1) ^ ek[42];
    const uint32_t o3 = enc_last(lds, lo, s3, s0, s1, s2) ^ ek[43];
    s0 = o0; s1 = o1; s2 = o2; s3 = o3;
}

// ---- decryption (_decryptBlock, cyr_rijndael.cpp:708-774) -----------------
// TL5 has LE bytes (14s, 9s, 13s, 11s); TL6/TL7/TL8 = rotl8/16/24 of it.
// Column j takes b0(u_j), b1(u_j-1), b2(u_j-2), b3(u_j-3) (inverse
// ShiftRows, cyr_rijndael.cpp:731-746).
// 160 KiB decrypt image: region 0 = TL5 | TL7, region 1 = TL6 | TL8 (TL6/TL8
// = rotl8 of TL5/TL7, made during the fill), so a middle-round column is
// tcol, as encrypt's (A/B vs the 128 KiB TL5|TL7 image with one rotation
// per column: same LDS cycles, -1.2 % time from the higher clock), and Si at
// 128 KiB in 128-B rows (32 slots): x << 7 | lane*4 | 128 KiB, built with one
// full-rate shift and one sel (addr_si).
__device__ __forceinline__ uint32_t dec_lo(uint32_t tid) { return ((tid & 31u) << 2) | 0x10000u; }
constexpr uint32_t kSiRowMask = 0x00007F80u;
template <int K>  // byte K of u
__device__ __forceinline__ uint32_t addr_si(uint32_t u, uint32_t lsi) {
    if constexpr (K == 0) return sel(kSiRowMask, u << 7, lsi);
    else return sel(kSiRowMask, u >> (8 * K - 7), lsi);
}
__device__ __forceinline__ uint32_t dec_last(const char* lds, uint32_t lsi, uint32_t x0, uint32_t x1, uint32_t x2,
                                             uint32_t x3) {
    const uint32_t l0 = ld(lds, addr_si<0>(x0, lsi));
    const uint32_t l1 = ld(lds, addr_si<1>(x1, lsi));
    const uint32_t l2 = ld(lds, addr_si<2>(x2, lsi));
    const uint32_t l3 = ld(lds, addr_si<3>(x3, lsi));
    return merge4(l0, l1, l2, l3);
}
__device__ __forceinline__ void fill_dec_image(uint32_t* lds, const uint32_t* __restrict__ t) {
    uint4* l4 = reinterpret_cast<uint4*>(lds);
    for (int q = threadIdx.x; q < 8192; q += blockDim.x) {  // two 64 KiB T regions
        const int region = q >> 12, half = (q >> 3) & 1, row = (q >> 4) & 255;
        uint32_t v = t[256 * half + row];
        if (region) v = rotl8(v);
        l4[q] = make_uint4(v, v, v, v);
    }
    for (int q = threadIdx.x; q < 2048; q += blockDim.x) {  // Si: 256 rows x 128 B
        const uint32_t v = t[512 + (q >> 3)];
        l4[8192 + q] = make_uint4(v, v, v, v);
    }
}
// prio_feedback counters of the decrypt workgroups: the 160 KiB image leaves
// no LDS word free, so they live in global memory (one per workgroup, reset by
// it at start; a collision between concurrent launches only blurs priorities).
constexpr uint32_t kLeadSlots = 4096;
__device__ unsigned int g_dec_lead[kLeadSlots];

// Decrypts N independent blocks together (N-way ILP per LDS round trip) and
// returns D(c[n]) ^ prev[n] in prev[n] (CBC, cyr_rijndael.cpp:625-630).
template <int N>
__device__ __forceinline__ void dec_cbc(const char* lds, uint32_t lo, const uint32_t* __restrict__ dk,
                                        const uint4 (&c)[N], uint4 (&prev)[N]) {
    uint32_t s[N][4];
#pragma unroll
    for (int n = 0; n < N; n++) {
        s[n][0] = c[n].x ^ dk[0]; s[n][1] = c[n].y ^ dk[1];
        s[n][2] = c[n].z ^ dk[2]; s[n][3] = c[n].w ^ dk[3];
    }
#pragma unroll
    for (int r = 1; r < 10; r++) {
        uint32_t t[N][4];
#pragma unroll
        for (int n = 0; n < N; n++) {
            t[n][0] = tcol(lds, lo, s[n][0], s[n][3], s[n][2], s[n][1], dk[4 * r + 0]);
            t[n][1] = tcol(lds, lo, s[n][1], s[n][0], s[n][3], s[n][2], dk[4 * r + 1]);
            t[n][2] = tcol(lds, lo, s[n][2], s[n][1], s[n][0], s[n][3], dk[4 * r + 2]);
            t[n][3] = tcol(lds, lo, s[n][3], s[n][2], s[n][1], s[n][0], dk[4 * r + 3]);
        }
#pragma unroll
        for (int n = 0; n < N; n++)
#pragma unroll
            for (int j = 0; j < 4; j++) s[n][j] = t[n][j];
    }
#pragma unroll
    for (int n = 0; n < N; n++) {
        const uint32_t lsi = (lo & 0xFFu) | 0x20000u;  // lane bits | 128 KiB (Si image)
        prev[n] = make_uint4(xor3(dec_last(lds, lsi, s[n][0], s[n][3], s[n][2], s[n][1]), dk[40], prev[n].x),
                             xor3(dec_last(lds, lsi, s[n][1], s[n][0], s[n][3], s[n][2]), dk[41], prev[n].y),
                             xor3(dec_last(lds, lsi, s[n][2], s[n][1], s[n][0], s[n][3]), dk[42], prev[n].z),
                             xor3(dec_last(lds, lsi, s[n][3], s[n][2], s[n][1], s[n][0]), dk[43], prev[n].w));
    }
}

// Key index of payload p (cyaes.h): key_idx[p] | p / ppk | 0, clamped.
__device__ __forceinline__ uint32_t key_index(const KeySel& ks, uint64_t p, uint64_t npayloads, bool active,
                                              uint32_t* status) {
    if (!active) return 0;
    uint32_t kid = ks.key_idx ? LD4(ks.key_idx + p, ext(ks.key_idx, 4 * npayloads))
                              : (ks.ppk.d ? fastdiv((uint32_t)p, ks.ppk) : 0u);
    if (kid >= ks.nkeys) {
        atomicOr(status, 1u);
        kid = ks.nkeys - 1;
    }
    return kid;
}

__device__ __forceinline__ uint32_t rl63(uint32_t v) { return __builtin_amdgcn_readlane(v, 63); }

// Loads one 44-word half of schedule `kid` (half 0: ek, 1: dk; wave-uniform
// address) into SGPRs.  The table is only read by the kernels, but the
// compiler cannot prove the batch's stores do not alias it, so it would
// otherwise keep the words in VGPRs or re-load them with vector loads inside
// the block loop.
__device__ __forceinline__ void load_sched(const KeySel& ks, uint32_t kid, int half, uint32_t (&k)[44]) {
    const uint32_t* p = ks.table + (uint64_t)kid * kSchedWords + 44 * half;
    const Ext e = key_ext(ks);
#pragma unroll
    for (int i = 0; i < 11; i++) {
        const uint4 v = LD16(p + 4 * i, e);
        k[4 * i + 0] = __builtin_amdgcn_readfirstlane(v.x);
        k[4 * i + 1] = __builtin_amdgcn_readfirstlane(v.y);
        k[4 * i + 2] = __builtin_amdgcn_readfirstlane(v.z);
        k[4 * i + 3] = __builtin_amdgcn_readfirstlane(v.w);
    }
}

// Progress-feedback wave priority.  The SQ serves the oldest ready wave
// first, so under LDS saturation the 16 waves of a workgroup would finish
// staggered (measured with CYAES_CLOCK_PROBE: wave 0 at ~55 % of the kernel
// time, wave 15 at 100 %) and the tail would run with 4 waves/CU, far below
// the LDS gather peak.  Each wave publishes its step count to an LDS max; a
// wave trailing the block's leader by d steps runs at priority min(d / div, 3).
// The waves then finish together (probe: within 1 %); -7.5 % encrypt and -8 %
// decrypt time on config C (tools/ab.py).  Lockstepping the waves with
// s_barrier instead was measured worse (encrypt +5 %, decrypt -4 %).
__device__ __forceinline__ void prio_feedback(uint32_t* lead, uint32_t step, uint32_t div) {
    // first active lane publishes (lane 0 may be masked off in a waterfall)
    const uint32_t fl = (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec());
    uint32_t m = 0;
    if (__lane_id() == fl) m = atomicMax(lead, step);
    m = __builtin_amdgcn_readfirstlane(m);
    step = __builtin_amdgcn_readfirstlane(step);  // keeps d scalar: the branches below must be uniform jumps,
    const uint32_t d = m > step ? (m - step) / div : 0u;  // not exec-masked (s_setprio ignores exec)
    if (d >= 3) __builtin_amdgcn_s_setprio(3);
    else if (d == 2) __builtin_amdgcn_s_setprio(2);
    else if (d == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}
constexpr uint32_t kEncPrioDiv = 4;  // steps = 8-block chunks (A/B: 1, 2, 4, 8 -> 4 best)
constexpr uint32_t kDecPrioDiv = 8;  // steps = 64*kDecRows-block rows (A/B: 4, 8, 16 -> 8)

__device__ __forceinline__ uint4 default_iv() { return make_uint4(kIv0, kIv1, kIv2, kIv3); }

#if CYAES_CLOCK_PROBE
// Variant builds only (make probe): per-wave shader cycles (s_memtime) and
// wall ticks (s_memrealtime, 100 MHz per tools/clockcal.hip) over the kernel
// body, summed per kernel kind into g_probe and read by cyaes_debug_probe()
// (bench.py and tools/ab.py print the clock).
__device__ unsigned long long g_probe[2][4];  // [enc, dec] x {cycles, ticks, waves, max ticks}
struct ClockProbe {
    uint64_t t0, r0;
    int kind;
    __device__ explicit ClockProbe(int k) : t0(__builtin_amdgcn_s_memtime()), r0(__builtin_amdgcn_s_memrealtime()), kind(k) {}
    __device__ ~ClockProbe() {
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&g_probe[kind][0], (unsigned long long)(t1 - t0));
            atomicAdd(&g_probe[kind][1], (unsigned long long)(r1 - r0));
            atomicAdd(&g_probe[kind][2], 1ull);
            atomicMax(&g_probe[kind][3], (unsigned long long)(r1 - r0));
        }
    }
};
#define CLOCK_PROBE(k) ClockProbe clock_probe_(k)
#else
#define CLOCK_PROBE(k)
#endif

// In-place batches: every load of a step must have returned before the step's
// first store (a lane's previous-block load reads a neighbour's block).
__device__ __forceinline__ void drain_loads() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---- CBC encrypt: one lane per payload chain (cyr_rijndael.cpp:588-609) ----
// RUNS (uniform batches of short payloads, no IV arrays): a lane's work item
// is a run of a.run consecutive payloads, contiguous in memory, encrypted as
// one block stream whose chain restarts at DefaultIV every bpp blocks
// (relay_local.cpp:206 passes no IV, so every payload is its own chain).  The
// next-chunk prefetch then never stops at a payload boundary: a lane of
// config B (1,472-B payloads) streams 368 blocks instead of four 92-block
// payloads, each of which started on an exposed load and ended in a 4-block
// tail.  The restart test is on wave-uniform block counters (scalar).
// SESS (uniform batches keyed by sessions of payloads_per_key payloads that
// are whole waves long, config D): a wave's work items all lie in one session,
// so its key comes from the scalar position, per wave, in SGPRs -- the
// unkeyed code path, no per-lane key index and no waterfall.  The grid has a
// lane per work item (not persistent).
template <bool RAGGED, bool KEYED, bool RUNS, bool SESS>
__global__ __launch_bounds__(kEncThreads, 1) void k_encrypt(EncArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_words[kEncLdsWords];
    fill_region(lds_words, a.tables, a.tables + 512, blockDim.x);              // TL1 | TL3
    fill_region(lds_words + 16384, a.tables + 256, a.tables + 768, blockDim.x);  // TL2 | TL4
    __shared__ uint32_t lead;  // prio_feedback
    if (threadIdx.x == 0) lead = 0;
    uint32_t prog = 0;
    __syncthreads();
    CLOCK_PROBE(0);
    const char* lds = reinterpret_cast<const char*>(lds_words);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lo = ((threadIdx.x & 31u) << 2) | 0x10000u;
    // Block size: kEncThreads for big batches; fewer for small ones, so that
    // few chains spread over many CUs (cyaes_runtime.cpp, wave_shape).
    const uint64_t wstride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t wbase0 = (uint64_t)blockIdx.x * blockDim.x + __builtin_amdgcn_readfirstlane(threadIdx.x & ~63u);
    const Ext iv_in_e = iv_ext(a.iv_in, a.npayloads), iv_out_e = iv_ext(a.iv_out, a.npayloads);
    const uint32_t R = RUNS ? a.run : 1u;  // payloads per work item
    const uint32_t bpp = a.payload_bytes >> 4;
    const uint64_t nwork = RUNS ? (a.npayloads + R - 1) / R : a.npayloads;
    uint32_t ek[44];
    // One schedule per wave, loaded before the loop: the whole batch's, or
    // (SESS) the wave's session's, from its scalar position.  A SESS grid covers
    // the batch in one pass (one work item per lane, the runtime sizes the
    // grid), so the loop body runs once.  Re-loading ek inside the loop instead
    // made the compiler schedule the round loop with 57 s_waitcnt per 160 LDS
    // reads against 44 (config D encrypt 1.11 ms against B's 1.09).
    if (SESS) load_sched(a.keys, wbase0 < nwork ? (uint32_t)(wbase0 * R / a.sess_payloads) : 0u, 0, ek);
    else if (!KEYED) load_sched(a.keys, 0, 0, ek);

    for (uint64_t wbase = wbase0; wbase < nwork; wbase += wstride) {
        const uint64_t w = wbase + lane;
        const bool active = w < nwork;
        const uint64_t p = RUNS ? w * R : w;  // (first) payload of the work item
        uint64_t off;
        uint32_t nb;
        if (RAGGED) {
            off = active ? LD8(a.offsets + p, ext(a.offsets, 8 * a.npayloads)) : 0;
            nb = active ? (LD4(a.nbytes + p, ext(a.nbytes, 4 * a.npayloads)) >> 4) : 0;
        } else {
            off = p * (uint64_t)a.payload_bytes;
            nb = active ? (RUNS ? (uint32_t)min<uint64_t>(R, a.npayloads - p) * bpp : bpp) : 0;
        }
        // RUNS + KEYED: the runtime makes runs divide payloads_per_key, so the run is one session
        const uint32_t kid = KEYED ? key_index(a.keys, p, a.npayloads, active, a.status) : 0u;
        bool pending = active;
        while (true) {  // waterfall over the distinct keys of this wave
            const uint64_t m = __ballot(pending);
            if (m == 0) break;
            const uint32_t ku = KEYED ? __builtin_amdgcn_readlane(kid, __builtin_ctzll(m)) : 0u;
            if (pending && (!KEYED || kid == ku)) {
                pending = false;
                if (KEYED) load_sched(a.keys, ku, 0, ek);
                uint4 c = a.iv_in ? LD16(a.iv_in + 16 * p, iv_in_e) : default_iv();
                const uint8_t* src = a.in + off;  // ragged: 4-B aligned
                uint8_t* dst = a.out + off;
                const Ext se = ext(src, 16ull * nb), de = ext(dst, 16ull * nb);  // this work item's bytes
                uint32_t nr = bpp;  // RUNS: block index of the next chain restart (a payload start)
                uint32_t i = 0;
                uint4 b[8];
                if (nb >= 8) {
#pragma unroll
                    for (int j = 0; j < 8; j++) b[j] = ldb<RAGGED>(src, j, se);
                }
                bool have_tail = false;  // b[8 - (nb - i), 8) already hold the last partial chunk
                for (; i + 8 <= nb; i += 8) {
                    const bool more = i + 16 <= nb;
                    const bool tail = !more && i + 8 < nb;  // partial last chunk
                    // Next chunk's loads in flight during this chunk's rounds (-8 %
                    // encrypt time).  One set of 8 loads for both cases: a partial
                    // last chunk loads the payload's last 8 blocks (its tail then
                    // sits at the top of bn).  With every bn[j] defined on this
                    // path the compiler no longer waits for this chunk's stores
                    // (s_waitcnt vmcnt(0)) before the next chunk's loads; it waits
                    // only for the loads (profiles/r02/ab_onepf.txt).
                    uint4 bn[8];
                    if (more || tail) {
                        const uint8_t* nsrc = src + 16ull * (more ? i + 8 : nb - 8);
#pragma unroll
                        for (int j = 0; j < 8; j++) bn[j] = ldb<RAGGED>(nsrc, j, se);
                    }
                    prio_feedback(&lead, ++prog, kEncPrioDiv);
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        if (RUNS && i + j == nr) {  // next payload of the run: a new chain
                            c = default_iv();
                            nr += bpp;
                        }
                        uint32_t s0 = xor3(c.x, b[j].x, ek[0]), s1 = xor3(c.y, b[j].y, ek[1]);
                        uint32_t s2 = xor3(c.z, b[j].z, ek[2]), s3 = xor3(c.w, b[j].w, ek[3]);
                        enc_block(lds, lo, ek, s0, s1, s2, s3);
                        c = make_uint4(s0, s1, s2, s3);
                        b[j] = c;
                    }
                    uint8_t* const dchunk = dst + 16ull * i;  // one address, immediate offsets (ragged too)
#pragma unroll
                    for (int j = 0; j < 8; j++) stb<RAGGED>(dchunk, j, b[j], de);  // (nt stores measured 3.6x slower)
                    if (more || tail) {
#pragma unroll
                        for (int j = 0; j < 8; j++) b[j] = bn[j];
                    }
                    have_tail = tail;
                }
                if (have_tail) {  // the tail's nb - i blocks sit in b[8 - (nb - i), 8): move them down to b[0]
#pragma unroll
                    for (int sft = 1; sft < 8; sft++) {
                        if (sft <= 8 - (int)(nb - i)) {
#pragma unroll
                            for (int j = 0; j < 7; j++) b[j] = b[j + 1];
                        }
                    }
                }
                for (; i < nb; i++) {  // partial last chunk: from b (prefetched) or loaded here
                    const uint4 v = have_tail ? b[0] : ldb<RAGGED>(src, i, se);
#pragma unroll
                    for (int j = 0; j < 7; j++) b[j] = b[j + 1];
                    if (RUNS && i == nr) {
                        c = default_iv();
                        nr += bpp;
                    }
                    uint32_t s0 = xor3(c.x, v.x, ek[0]), s1 = xor3(c.y, v.y, ek[1]);
                    uint32_t s2 = xor3(c.z, v.z, ek[2]), s3 = xor3(c.w, v.w, ek[3]);
                    enc_block(lds, lo, ek, s0, s1, s2, s3);
                    c = make_uint4(s0, s1, s2, s3);
                    stb<RAGGED>(dst, i, c, de);
                }
                if (a.iv_out) ST16(a.iv_out + 16 * p, iv_out_e, c);  // (RUNS: no IV arrays)
            }
        }
        if (SESS) break;  // one pass (above)
    }
}

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
        if (RAGGED) {
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

// ---- CBC decrypt, uniform contiguous batch: one lane per block ------------
// The batch is one array of nblocks blocks; payload boundaries every bpp
// blocks restart the chain at the IV.  Each wave owns the contiguous range
// [w*bpw, (w+1)*bpw) (bpw a multiple of 64*R) and walks it in steps of 64*R
// blocks: R rows of 64 lanes, decrypted together (R-way ILP).  BIG: bpp >= 64*R,
// so a step holds at most one payload start and needs no division.
// Per-wave walk state of k_decrypt_flat (kept in registers: passed by value
// and returned, never through memory).
struct FlatPos {
    uint64_t bp;    // payload of the step's first block
    uint32_t bpos;  // its position in the payload
};

// Position of row k's block in its payload (r) and the payload index (p).
template <bool BIG>
__device__ __forceinline__ void flat_position(const DecArgs& a, FlatPos ps, uint32_t lane, int k, uint32_t& r,
                                              uint64_t& p) {
    const uint32_t lpos = ps.bpos + 64 * k + lane;
    const uint32_t bpp = a.bpp.d;
    if (BIG) {
        r = min(lpos, lpos - bpp);
        p = ps.bp + (lpos >= bpp ? 1 : 0);
    } else {
        const uint32_t q = fastdiv(lpos, a.bpp);
        r = lpos - q * bpp;
        p = ps.bp + q;
    }
}

// v (lane l-1) for lanes 1..63, old for lane 0: DPP wave_shr:1.
__device__ __forceinline__ uint32_t shr1(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint4 shr1(uint4 v, uint4 old) {
    return make_uint4(shr1(v.x, old.x), shr1(v.y, old.y), shr1(v.z, old.z), shr1(v.w, old.w));
}

// Loads the R rows of the step at `base` (c); partial steps also load each
// block's predecessor (pv), full steps take it from the neighbour lane.
// FULL: all 64*R blocks are in range (every step but possibly the batch's
// last), so loads are unguarded and use immediate offsets off one lane pointer.
template <bool FULL>
__device__ __forceinline__ void flat_load(const DecArgs& a, uint32_t lane, uint64_t base, uint64_t end,
                                          uint4 (&c)[kDecRows], uint4 (&pv)[kDecRows]) {
    constexpr int R = kDecRows;
    const Ext ie = ext(a.in, 16 * a.nblocks);
    if (FULL) {
        const uint8_t* g0 = a.in + 16 * (base + lane);
#pragma unroll
        for (int k = 0; k < R; k++) c[k] = LD16(g0 + 1024 * k, ie);
        // pv comes from the neighbour lane in flat_step (DPP), not from memory
    } else {  // last, partial step of the batch: clamp reads into range
#pragma unroll
        for (int k = 0; k < R; k++) {
            const uint64_t g = min(base + 64 * k + lane, end - 1);
            c[k] = LD16(a.in + 16 * g, ie);
            // The predecessor of block g (lane 0 of row 0 reads its own block:
            // the carry replaces it).  Block 0 has none: a 1-block batch (end
            // == 1) clamps every lane to g = 0, and g - 1 would read 16 B before
            // the buffer (r02 fault hunt, VERDICT r02 "What's weak" 1).  Block
            // 0 is a payload start, so its pv is the IV in flat_step anyway.
            const uint64_t back = (k == 0 && lane == 0) ? 0u : 1u;
            pv[k] = LD16(a.in + 16 * (g >= back ? g - back : 0u), ie);
        }
    }
}

template <bool KEYED, bool BIG, bool FULL>
__device__ __forceinline__ uint4 flat_step(const DecArgs& a, const char* lds, uint32_t lo, uint32_t lane,
                                           uint64_t base, uint64_t end, FlatPos ps, uint4 carry,
                                           uint32_t (&dk0)[44], uint32_t& dk_id, const uint4 (&c)[kDecRows],
                                           uint4 (&pv)[kDecRows]) {
    constexpr int R = kDecRows;
    const Ext oe = ext(a.out, 16 * a.nblocks);
    const Ext iv_in_e = iv_ext(a.iv_in, a.npayloads), iv_out_e = iv_ext(a.iv_out, a.npayloads);
    if (FULL) {
        // Predecessor blocks from the neighbour lane (DPP wave_shr:1), lane 0's
        // from the row before (or the carry): no second load of C[i-1]
        // (A/B: -4.8 % decrypt time vs the load at offset -16).  Every load of
        // the step is then the lane's own block, which its store needs anyway,
        // so in-place steps need no drain.
        pv[0] = shr1(c[0], carry);
#pragma unroll
        for (int k = 1; k < R; k++)
            pv[k] = shr1(c[k], make_uint4(rl63(c[k - 1].x), rl63(c[k - 1].y), rl63(c[k - 1].z), rl63(c[k - 1].w)));
    } else {
        if (lane == 0) pv[0] = carry;
        if (a.inplace) drain_loads();  // pv loads read neighbours' blocks
    }
    // Chain restarts at payload starts inside this step.
    if (BIG) {
        const uint32_t fo = ps.bpos == 0 ? 0u : a.bpp.d - ps.bpos;  // offset of the payload start, if < 64R
        // On a partial last step the "next payload" may start at or past the
        // batch's end: then it does not exist, and iv_in[pf] would read 16 B
        // past the IV array (VERDICT r02 "What's weak" 1).
        if (fo < 64u * R && (FULL || base + fo < end)) {
            const uint64_t pf = ps.bp + (ps.bpos == 0 ? 0 : 1);
            const uint4 ivv = a.iv_in ? LD16(a.iv_in + 16 * pf, iv_in_e) : default_iv();
#pragma unroll
            for (int k = 0; k < R; k++)
                if ((fo >> 6) == (uint32_t)k && lane == (fo & 63u)) pv[k] = ivv;
        }
    } else {
#pragma unroll
        for (int k = 0; k < R; k++) {
            uint32_t r;
            uint64_t p;
            flat_position<BIG>(a, ps, lane, k, r, p);
            if (r == 0) {
                const bool valid = FULL || base + 64 * k + lane < end;
                pv[k] = (a.iv_in && valid) ? LD16(a.iv_in + 16 * p, iv_in_e) : default_iv();
            }
        }
    }
    if (a.iv_out) {  // final chain block of each payload ending in this step
#pragma unroll
        for (int k = 0; k < R; k++) {
            uint32_t r;
            uint64_t p;
            flat_position<BIG>(a, ps, lane, k, r, p);
            if (r == a.bpp.d - 1 && (FULL || base + 64 * k + lane < end)) ST16(a.iv_out + 16 * p, iv_out_e, c[k]);
        }
    }
    uint4 d[R];
#pragma unroll
    for (int k = 0; k < R; k++) d[k] = pv[k];
    if (!KEYED) {
        dec_cbc<R>(lds, lo, dk0, c, d);  // all R rows per LDS round trip (A/B: ~1% over 2 rows)
    } else {
        uint32_t kid[R];
        bool valid[R];
#pragma unroll
        for (int k = 0; k < R; k++) {
            uint32_t r;
            uint64_t p;
            flat_position<BIG>(a, ps, lane, k, r, p);
            valid[k] = FULL || base + 64 * k + lane < end;
            kid[k] = key_index(a.keys, p, a.npayloads, valid[k], a.status);
        }
        // Sessions are contiguous runs of payloads (config D: 256 x 92 blocks),
        // so nearly every full step has one key: decrypt all R rows together
        // under it (R-way ILP), as the unkeyed path does.  Otherwise fall back
        // to a per-row waterfall over the keys present.
        const uint32_t k0 = __builtin_amdgcn_readfirstlane(kid[0]);
        bool same = true;
#pragma unroll
        for (int k = 0; k < R; k++) same = same && kid[k] == k0;
        const bool uniform = FULL && __ballot(!same) == 0;
        if (uniform) {
            // dk0 keeps the last session's schedule (SGPRs) across steps: a
            // session spans ~92 steps in config D
            if (k0 != dk_id) {
                load_sched(a.keys, k0, 1, dk0);
                dk_id = k0;
            }
            dec_cbc<R>(lds, lo, dk0, c, d);
        } else {
#pragma unroll
            for (int k = 0; k < R; k++) {
                bool pending = valid[k];
                while (true) {  // waterfall over the distinct keys of this row
                    const uint64_t m = __ballot(pending);
                    if (m == 0) break;
                    const uint32_t ku = __builtin_amdgcn_readlane(kid[k], __builtin_ctzll(m));
                    if (pending && kid[k] == ku) {
                        pending = false;
                        uint32_t dk[44];
                        load_sched(a.keys, ku, 1, dk);
                        const uint4 cc[1] = {c[k]};
                        uint4 dd[1] = {d[k]};
                        dec_cbc<1>(lds, lo, dk, cc, dd);
                        d[k] = dd[0];
                    }
                }
            }
        }
    }
    if (FULL) {
        uint8_t* o0 = a.out + 16 * (base + lane);
#pragma unroll
        for (int k = 0; k < R; k++) ST16(o0 + 1024 * k, oe, d[k]);
    } else {
#pragma unroll
        for (int k = 0; k < R; k++)
            if (base + 64 * k + lane < end) ST16(a.out + 16 * (base + 64 * k + lane), oe, d[k]);
    }
    return make_uint4(rl63(c[R - 1].x), rl63(c[R - 1].y), rl63(c[R - 1].z), rl63(c[R - 1].w));  // next carry
}

// SESS: sessions of payloads_per_key payloads that are whole steps long
// (a.sess_blocks, a multiple of 64 * R; config D: 256 x 92 blocks): no step
// straddles two sessions, so the unkeyed step runs under a schedule chosen per
// step from the scalar block position, and no lane computes a key index.
template <bool KEYED, bool BIG, bool SESS>
__global__ __launch_bounds__(kDecThreads, 1) void k_decrypt_flat(DecArgs a) {
    constexpr int R = kDecRows;
    __shared__ __attribute__((aligned(16))) uint32_t lds_words[kDecLdsWords];
    fill_dec_image(lds_words, a.tables);
    unsigned int* leadp = &g_dec_lead[blockIdx.x % kLeadSlots];
    if (threadIdx.x == 0) *leadp = 0;
    uint32_t prog = 0;
    __syncthreads();
    CLOCK_PROBE(1);
    const uint64_t wave =
        (uint64_t)blockIdx.x * (kDecThreads / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t begin = wave * a.blocks_per_wave;
    if (begin >= a.nblocks) return;
    const char* lds = reinterpret_cast<const char*>(lds_words);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lo = dec_lo(threadIdx.x);
    const uint64_t end = min(begin + a.blocks_per_wave, a.nblocks);
    FlatPos ps;
    ps.bp = begin / a.bpp.d;
    ps.bpos = (uint32_t)(begin - ps.bp * a.bpp.d);
    uint4 carry = make_uint4(0, 0, 0, 0);  // C[base-1]
    if (ps.bpos != 0)  // (begin >= 1 here)
        carry = a.boundary ? LD16(a.boundary + wave, ext(a.boundary, 16ull * gridDim.x * (kDecThreads / 64)))
                           : LD16(a.in + 16 * (begin - 1), ext(a.in, 16 * a.nblocks));
    uint32_t dk0[44];
    uint32_t dk_id = 0;  // KEYED: session whose schedule dk0 holds (~0u: none yet)
    uint32_t sess = 0;   // SESS: session of the current step; it ends at block sess_next
    uint64_t sess_next = 0;
    if (SESS) {
        sess = (uint32_t)(begin / a.sess_blocks);
        sess_next = (uint64_t)(sess + 1) * a.sess_blocks;
        load_sched(a.keys, sess, 1, dk0);
    } else if (!KEYED) {
        load_sched(a.keys, 0, 1, dk0);
    } else {
        dk_id = ~0u;
    }
    uint64_t base = begin;
    uint4 c[R], pv[R];
    if (base + 64 * R <= end) flat_load<true>(a, lane, base, end, c, pv);
    for (; base + 64 * R <= end; base += 64 * R) {
        if (SESS && base >= sess_next) {  // (make_keysel checked every session is in the table)
            sess++;
            sess_next += a.sess_blocks;
            load_sched(a.keys, sess, 1, dk0);
        }
        // (Issuing the next step's loads before this step's rounds measured ~1 %
        // slower: the LDS binds, and the other 15 waves hide the loads.)
        carry = flat_step<KEYED, BIG, true>(a, lds, lo, lane, base, end, ps, carry, dk0, dk_id, c, pv);
        if (base + 128 * R <= end) flat_load<true>(a, lane, base + 64 * R, end, c, pv);
        prio_feedback(leadp, ++prog, kDecPrioDiv);
        ps.bpos += a.step_r;
        ps.bp += a.step_q;
        if (ps.bpos >= a.bpp.d) { ps.bpos -= a.bpp.d; ps.bp++; }
    }
    if (base < end) {
        if (SESS && base >= sess_next) load_sched(a.keys, sess + 1, 1, dk0);
        flat_load<false>(a, lane, base, end, c, pv);
        flat_step<KEYED, BIG, false>(a, lds, lo, lane, base, end, ps, carry, dk0, dk_id, c, pv);
    }
}

// ---- CBC decrypt, ragged batch: groups of payloads packed into wave rows ---
// A wave takes a group of G consecutive payloads (G <= 64, a.group) and
// walks their blocks as one flat sequence in steps of R rows x 64 lanes, as
// k_decrypt_flat does: a row holds the tail of one payload and the head of the
// next, so 1,472-B relay packets (92 blocks) fill the rows instead of leaving
// 164 of every 256 lanes idle (one wave per payload).  Lane j of the wave
// holds payload j's block count, offset and key; a row finds each lane's
// payload by a binary search over the group's block prefix (ds_bpermute),
// narrowed to the payloads that start inside the row (usually 0 or 1 step).
// The predecessor block is the neighbour lane's (DPP), or the IV where a
// payload starts, so in-place batches need no drain.
__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t src_lane) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}
__device__ __forceinline__ uint64_t bperm64(uint64_t v, uint32_t src_lane) {
    return (uint64_t)bperm((uint32_t)(v >> 32), src_lane) << 32 | bperm((uint32_t)v, src_lane);
}
// Lane l's value of v (l wave-uniform).  The builtin returns int: widen as
// unsigned, or a low word >= 2^31 sign-extends into the high word.
__device__ __forceinline__ uint64_t rlane64(uint64_t v, uint32_t l) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
    return (uint64_t)hi << 32 | lo;
}

template <bool KEYED>
__global__ __launch_bounds__(kDecThreads, 1) void k_decrypt_ragged(DecArgs a) {
    constexpr int R = kDecRows;
    __shared__ __attribute__((aligned(16))) uint32_t lds_words[kDecLdsWords];
    fill_dec_image(lds_words, a.tables);
    unsigned int* leadp = &g_dec_lead[blockIdx.x % kLeadSlots];
    if (threadIdx.x == 0) *leadp = 0;
    uint32_t prog = 0;
    __syncthreads();
    const char* lds = reinterpret_cast<const char*>(lds_words);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lo = dec_lo(threadIdx.x);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t wave0 =
        (uint64_t)blockIdx.x * (blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t G = a.group;
    const uint64_t ngroups = (a.npayloads + G - 1) / G;
    const Ext iv_in_e = iv_ext(a.iv_in, a.npayloads), iv_out_e = iv_ext(a.iv_out, a.npayloads);
    uint32_t dk0[44];
    uint32_t dk_id = ~0u;  // session whose schedule dk0 holds
    if (!KEYED) {
        load_sched(a.keys, 0, 1, dk0);
        dk_id = 0;
    }
    for (uint64_t grp = wave0; grp < ngroups; grp += nwaves) {
        const uint64_t p0 = grp * G;
        const uint32_t gn = (uint32_t)min<uint64_t>(G, a.npayloads - p0);
        const bool holder = lane < gn;
        const uint64_t ph = p0 + lane;
        const uint32_t nbh = holder ? LD4(a.nbytes + ph, ext(a.nbytes, 4 * a.npayloads)) >> 4 : 0u;
        const uint64_t offh = holder ? LD8(a.offsets + ph, ext(a.offsets, 8 * a.npayloads)) : 0ull;
        const uint32_t kidh = KEYED ? key_index(a.keys, ph, a.npayloads, holder, a.status) : 0u;
        if (holder && nbh == 0 && a.iv_out)  // empty chain: the IV comes back unchanged
            ST16(a.iv_out + 16 * ph, iv_out_e, a.iv_in ? LD16(a.iv_in + 16 * ph, iv_in_e) : default_iv());
        // Regular group: every payload has nb0 >= 64 blocks and the offsets are
        // equally strided (a relay stream of MTU-sized packets: payload p at
        // o + p * packet size).  Then each lane walks its own (payload, block)
        // position -- +64 blocks a row, at most one payload boundary -- with no
        // per-row ballots, scalar reads or search (profiles/r02/ab_ragged_regular.txt).
        const uint32_t nb0 = __builtin_amdgcn_readfirstlane(nbh);  // lane 0 holds a payload
        const uint64_t off0 = rlane64(offh, 0);
        const uint64_t ostr = gn > 1 ? rlane64(offh, 1) - off0 : 0;
        const bool regular =
            nb0 >= 64 && __ballot(holder && (nbh != nb0 || offh != off0 + (uint64_t)lane * ostr)) == 0;
        uint32_t jt = 0, rt = lane - 64u;  // regular: this lane's payload and block; the first row adds 64
        // Inclusive prefix of the group's block counts (64-bit: payloads may be up to 2^28 blocks).
        uint64_t incl = nbh;
        if (!regular) {
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint64_t t = (uint64_t)__shfl_up((unsigned int)(incl >> 32), d) << 32 |
                                   __shfl_up((unsigned int)incl, d);
                if (lane >= (uint32_t)d) incl += t;
            }
        }
        const uint64_t bsh = incl - nbh;  // first flat block of payload `lane`
        const uint64_t total = regular ? (uint64_t)gn * nb0 : rlane64(incl, 63);  // lanes >= gn add 0
        uint4 carry = make_uint4(0, 0, 0, 0);
        for (uint64_t base = 0; base < total; base += 64 * R) {
            uint4 c[R], pv[R];
            uint32_t jr[R], rr[R];
            uint64_t orow[R];
            bool valid[R];
#pragma unroll
            for (int k = 0; k < R; k++) {
                if (regular) {
                    rt += 64;
                    if (rt >= nb0) rt -= nb0, jt++;
                    valid[k] = jt < gn;
                    rr[k] = rt;
                    jr[k] = jt;
                    orow[k] = off0 + (uint64_t)jt * ostr + 16ull * rt;
                    continue;
                }
                const uint64_t rlo = base + 64 * k;
                const uint64_t g = rlo + lane;
                valid[k] = g < total;
                // Payloads present in the row: jlo (holds rlo) .. jhi (holds the row's last valid block).
                const uint64_t rhi = min(rlo + 63u, total - 1u);
                const uint64_t mlo = __ballot(holder && bsh <= rlo);
                const uint64_t mhi = __ballot(holder && bsh <= rhi);
                uint32_t j = mlo ? 63u - (uint32_t)__builtin_clzll(mlo) : 0u;
                const uint32_t jhi = mhi ? 63u - (uint32_t)__builtin_clzll(mhi) : 0u;
                if (jhi == j) {  // the whole row in one payload (always for large payloads): scalar reads
                    const uint64_t bs = rlane64(bsh, j);
                    const uint64_t of = rlane64(offh, j);
                    rr[k] = (uint32_t)(g - bs);  // < 2^28: within one payload
                    orow[k] = of + 16ull * rr[k];
                } else if (jhi == j + 1) {  // two payloads (most rows of MTU-sized packets): scalar reads, one select
                    const uint64_t bs0 = rlane64(bsh, j), bs1 = rlane64(bsh, jhi);
                    const uint64_t of0 = rlane64(offh, j), of1 = rlane64(offh, jhi);
                    const bool second = g >= bs1;
                    rr[k] = (uint32_t)(g - (second ? bs1 : bs0));
                    orow[k] = (second ? of1 : of0) + 16ull * rr[k];
                    j = second ? jhi : j;
                } else {  // largest j in [jlo, jhi] with bs_j <= g (an empty payload never wins)
                    uint32_t hi = jhi;
                    const int steps = 32 - __builtin_clz(jhi - j);
                    for (int st = 0; st < steps; st++) {
                        const uint32_t mid = (j + hi + 1) >> 1;
                        if (bperm64(bsh, mid) <= g) j = mid;
                        else hi = mid - 1;
                    }
                    rr[k] = (uint32_t)(g - bperm64(bsh, j));
                    orow[k] = bperm64(offh, j) + 16ull * rr[k];
                }
                jr[k] = j;
            }
            // Extent of each row's payload (bounds build only: a lane's payload
            // j's bytes; an invalid lane loads row 0 lane 0's block, below).
            Ext re[R];
            const uint32_t j00 = __builtin_amdgcn_readlane(jr[0], 0);  // (not readfirstlane: exec may be partial)
#pragma unroll
            for (int k = 0; k < R; k++) {
                if constexpr (CYAES_BOUNDS_CHECK) {
                    const uint32_t j = valid[k] ? jr[k] : j00;
                    re[k] = ext(a.in + bperm64(offh, j), 16ull * bperm(nbh, j));
                } else {
                    re[k] = Ext{nullptr, nullptr};
                }
            }
            // All four rows' loads back to back, unconditionally: a lane past the
            // group's end loads row 0 lane 0's block (always valid) and its result
            // is never used (a valid lane's predecessor is valid).  A load under
            // `valid ? load : 0` joined the branches with a vmcnt(0) wait per row.
            const uint64_t safe = rlane64(orow[0], 0);
#pragma unroll
            for (int k = 0; k < R; k++) c[k] = LD16U(a.in + (valid[k] ? orow[k] : safe), re[k]);
            // The progress atomic (a global word: the decrypt image fills the LDS) goes
            // out after the step's loads, so its round trip overlaps theirs instead of
            // delaying them (A/B: -1 % on relay streams, profiles/r02/ab_ragged_prio_late.txt).
            prio_feedback(leadp, ++prog, kDecPrioDiv);
            pv[0] = shr1(c[0], carry);
#pragma unroll
            for (int k = 1; k < R; k++)
                pv[k] = shr1(c[k], make_uint4(rl63(c[k - 1].x), rl63(c[k - 1].y), rl63(c[k - 1].z), rl63(c[k - 1].w)));
#pragma unroll
            for (int k = 0; k < R; k++) {
                const uint64_t p = p0 + jr[k];
                if (valid[k] && rr[k] == 0) pv[k] = a.iv_in ? LD16(a.iv_in + 16 * p, iv_in_e) : default_iv();
                if (a.iv_out) {  // (uniform branch: every lane runs the bpermute; one from an inactive lane reads 0)
                    const uint32_t nbj = regular ? nb0 : bperm(nbh, jr[k]);
                    if (valid[k] && rr[k] + 1 == nbj) ST16(a.iv_out + 16 * p, iv_out_e, c[k]);
                }
            }
            if (!KEYED) {
                dec_cbc<R>(lds, lo, dk0, c, pv);
            } else {
                uint32_t kid[R];
#pragma unroll
                for (int k = 0; k < R; k++) kid[k] = bperm(kidh, jr[k]);
                const uint32_t k0 = __builtin_amdgcn_readfirstlane(kid[0]);  // lane 0 of row 0 is valid
                bool same = true;
#pragma unroll
                for (int k = 0; k < R; k++) same = same && (!valid[k] || kid[k] == k0);
                if (__ballot(!same) == 0) {  // one session in the whole step (the common case)
                    if (k0 != dk_id) {
                        load_sched(a.keys, k0, 1, dk0);
                        dk_id = k0;
                    }
                    dec_cbc<R>(lds, lo, dk0, c, pv);
                } else {
#pragma unroll
                    for (int k = 0; k < R; k++) {
                        bool pending = valid[k];
                        while (true) {  // waterfall over the sessions of this row
                            const uint64_t m = __ballot(pending);
                            if (m == 0) break;
                            const uint32_t ku = __builtin_amdgcn_readlane(kid[k], __builtin_ctzll(m));
                            if (pending && kid[k] == ku) {
                                pending = false;
                                uint32_t dk[44];
                                load_sched(a.keys, ku, 1, dk);
                                const uint4 cc[1] = {c[k]};
                                uint4 dd[1] = {pv[k]};
                                dec_cbc<1>(lds, lo, dk, cc, dd);
                                pv[k] = dd[0];
                            }
                        }
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < R; k++) {
                Ext we = re[k];
                if constexpr (CYAES_BOUNDS_CHECK) we = ext(a.out + (we.lo - a.in), we.hi - we.lo);
                if (valid[k]) ST16U(a.out + orow[k], we, pv[k]);
            }
            carry = make_uint4(rl63(c[R - 1].x), rl63(c[R - 1].y), rl63(c[R - 1].z), rl63(c[R - 1].w));
        }
    }
}

// In-place flat decrypt: snapshot C[begin-1] of every wave range before any
// wave overwrites it.
__global__ void k_boundary_snapshot(const uint4* in, uint64_t nblocks, uint64_t bpw, uint64_t nwaves, Fastdiv bpp,
                                    uint4* boundary) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nwaves) return;
    const uint64_t begin = w * bpw;
    if (begin == 0 || begin >= nblocks) return;
    if (begin % bpp.d != 0)
        ST16(boundary + w, ext(boundary, 16 * nwaves), LD16(in + (begin - 1), ext(in, 16 * nblocks)));
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

hipError_t launch_encrypt(const EncArgs& a, int grid, int threads, hipStream_t stream) {
    const bool keyed = a.keys.key_idx != nullptr || a.keys.ppk.d != 0;
    const bool ragged = a.offsets != nullptr;
    const dim3 g(grid), b(threads);
    const bool runs = !ragged && a.run > 1;
    const bool sess = !ragged && a.sess_payloads != 0;  // keyed by whole-wave sessions: the unkeyed body per session
    if (ragged && keyed) hipLaunchKernelGGL((k_encrypt<true, true, false, false>), g, b, 0, stream, a);
    else if (ragged) hipLaunchKernelGGL((k_encrypt<true, false, false, false>), g, b, 0, stream, a);
    else if (sess && runs) hipLaunchKernelGGL((k_encrypt<false, false, true, true>), g, b, 0, stream, a);
    else if (sess) hipLaunchKernelGGL((k_encrypt<false, false, false, true>), g, b, 0, stream, a);
    else if (runs && keyed) hipLaunchKernelGGL((k_encrypt<false, true, true, false>), g, b, 0, stream, a);
    else if (runs) hipLaunchKernelGGL((k_encrypt<false, false, true, false>), g, b, 0, stream, a);
    else if (keyed) hipLaunchKernelGGL((k_encrypt<false, true, false, false>), g, b, 0, stream, a);
    else hipLaunchKernelGGL((k_encrypt<false, false, false, false>), g, b, 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_encrypt_quad(const EncArgs& a, int grid, int threads, hipStream_t stream) {
    const bool keyed = a.keys.key_idx != nullptr || a.keys.ppk.d != 0;
    const bool ragged = a.offsets != nullptr;
    const dim3 g(grid), b(threads);
    if (ragged && keyed) hipLaunchKernelGGL((k_encrypt_quad<true, true>), g, b, 0, stream, a);
    else if (ragged) hipLaunchKernelGGL((k_encrypt_quad<true, false>), g, b, 0, stream, a);
    else if (keyed) hipLaunchKernelGGL((k_encrypt_quad<false, true>), g, b, 0, stream, a);
    else hipLaunchKernelGGL((k_encrypt_quad<false, false>), g, b, 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_decrypt_flat(const DecArgs& a, int grid, hipStream_t stream) {
    const bool keyed = a.keys.key_idx != nullptr || a.keys.ppk.d != 0;
    const bool big = a.bpp.d >= 64u * kDecRows;
    const dim3 g(grid), b(kDecThreads);
    const bool sess = a.sess_blocks != 0;  // keyed by step-aligned sessions: the unkeyed step per session
    if (sess && big) hipLaunchKernelGGL((k_decrypt_flat<false, true, true>), g, b, 0, stream, a);
    else if (sess) hipLaunchKernelGGL((k_decrypt_flat<false, false, true>), g, b, 0, stream, a);
    else if (keyed && big) hipLaunchKernelGGL((k_decrypt_flat<true, true, false>), g, b, 0, stream, a);
    else if (keyed) hipLaunchKernelGGL((k_decrypt_flat<true, false, false>), g, b, 0, stream, a);
    else if (big) hipLaunchKernelGGL((k_decrypt_flat<false, true, false>), g, b, 0, stream, a);
    else hipLaunchKernelGGL((k_decrypt_flat<false, false, false>), g, b, 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_decrypt_ragged(const DecArgs& a, int grid, int threads, hipStream_t stream) {
    const bool keyed = a.keys.key_idx != nullptr || a.keys.ppk.d != 0;
    if (keyed) hipLaunchKernelGGL(k_decrypt_ragged<true>, dim3(grid), dim3(threads), 0, stream, a);
    else hipLaunchKernelGGL(k_decrypt_ragged<false>, dim3(grid), dim3(threads), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_boundary_snapshot(const uint8_t* in, uint64_t nblocks, uint64_t blocks_per_wave, uint64_t nwaves,
                                    Fastdiv bpp, uint4* boundary, hipStream_t stream) {
    const int threads = 256;
    const int grid = (int)((nwaves + threads - 1) / threads);
    hipLaunchKernelGGL(k_boundary_snapshot, dim3(grid), dim3(threads), 0, stream,
                       reinterpret_cast<const uint4*>(in), nblocks, blocks_per_wave, nwaves, bpp, boundary);
    return hipGetLastError();
}

hipError_t launch_key_expand(const uint8_t* d_keys, uint32_t nkeys, const uint8_t* d_sbox, uint32_t* d_sched,
                             hipStream_t stream) {
    const int threads = 64;
    const int grid = (int)((nkeys + threads - 1) / threads);
    hipLaunchKernelGGL(k_key_expand, dim3(grid), dim3(threads), 0, stream, d_keys, nkeys, d_sbox, d_sched);
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
// Reads and clears the probe sums: out[8] = g_probe (enc, dec).
extern "C" int cyaes_debug_probe(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(cyaes::g_probe), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    static const unsigned long long zero[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(cyaes::g_probe), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif

#if CYAES_BOUNDS_CHECK
// Reads and clears the bounds record: out[4] = misses, first miss's source
// line in this file, its offset from the extent's start, the extent's size;
// then up to 8 (line, misses) pairs of the lines that missed in out[4..20).
extern "C" int cyaes_debug_bounds(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(cyaes::g_bounds), sizeof(unsigned long long) * 4) != hipSuccess) return -1;
    static unsigned int lines[cyaes::kBoundsLines];
    if (hipMemcpyFromSymbol(lines, HIP_SYMBOL(cyaes::g_bounds_lines), sizeof(lines)) != hipSuccess) return -1;
    for (int i = 4; i < 20; i++) out[i] = 0;
    for (uint32_t l = 0, k = 4; l < cyaes::kBoundsLines && k < 20; l++)
        if (lines[l]) out[k++] = l, out[k++] = lines[l];
    static const unsigned long long zero[4] = {};
    static const unsigned int zl[cyaes::kBoundsLines] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(cyaes::g_bounds_lines), zl, sizeof(zl)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(cyaes::g_bounds), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif
