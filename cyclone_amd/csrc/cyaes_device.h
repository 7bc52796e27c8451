// cyaes_device.h -- device code shared by the gfx950 kernel translation units
// (cyaes_kernels.hip, cyaes_enc_kernels.hip, cyaes_dec_kernels.hip): the
// access layer, LDS T-table lookups, the AES rounds, key schedules in SGPRs,
// progress-feedback priority.  Everything is TU-local (anonymous namespace):
// each translation unit has its own copy of the device globals (progress
// slots, the bounds record, the clock probe).  Each TU defines CYAES_TU
// (0, 1, 2) before including this header; see cyaes_kernels.hip for the design.
#pragma once

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
constexpr uint32_t kBoundsLines = 8192;    // misses per source position (line; header lines + 5000)
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
// Source position of an access: its line, + 5000 when the access is in this
// header (cyaes_debug_bounds adds 10000 x the translation unit).
constexpr bool in_header(const char* f) {
    const char* e = f;
    while (*e) e++;
    return e - f >= 2 && e[-2] == '.' && e[-1] == 'h';
}
#define AT(p, e, bytes) bchk((p), (e), (bytes), __LINE__ + (in_header(__FILE__) ? 5000u : 0u))
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
// no LDS word free, so they live in the launch's work words (DecArgs.work,
// one per workgroup, reset by it at start).
__device__ __forceinline__ uint32_t* dec_lead_word(uint32_t* work) { return work + kWorkLeadOff + blockIdx.x; }

// A kernel's own arguments in the kernarg segment (constant address space:
// scalar loads).  Read through an opaque copy of this pointer, a value is
// loaded where it is used instead of being held in an SGPR across loops.
template <typename T>
using KernArg = const __attribute__((address_space(4))) T*;

// The dynamic pool of a launch (DecArgs.dyn): tickets [0, ndyn) in kXcds
// contiguous pools of per_xcd, one per XCD.  A wave takes the next ticket of
// its current pool (first its own XCD's: the atomic stays among that XCD's
// waves) and, once that pool is exhausted, moves on to the next one, so an
// XCD that runs ahead takes work from the slower ones and the XCDs finish
// together.  Returns ndyn when every pool is exhausted (at most kXcds failed
// tries).  Measured (tools/atomicbench.hip, profiles/r04/atomicbench.jsonl):
// one counter for all 4,096 waves ~88 M tickets/s (a ticket per 2-step range
// asks ~190 M/s: the first dynamic decrypt ran 2x slower), one per XCD ~540 M/s,
// one per workgroup ~9.3 G/s.
__device__ __forceinline__ uint32_t dyn_ticket(uint32_t* work, uint32_t& pool, uint32_t per_xcd, uint32_t ndyn) {
    const uint32_t fl = (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec());
    for (uint32_t k = 0; k < kXcds; k++) {
        uint32_t t = 0;
        if (__lane_id() == fl) t = atomicAdd(work + kWorkCtrOff + 64 * pool, 1u);
        t = __builtin_amdgcn_readfirstlane(t);
        const uint32_t g = pool * per_xcd + t;
        if (t < per_xcd && g < ndyn) return g;
        pool = pool + 1 < kXcds ? pool + 1 : 0;
    }
    return ndyn;
}
__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg(20 | (31 << 11)) % kXcds; }  // HW_REG_XCC_ID

// Decrypts N independent blocks together (N-way ILP per LDS round trip) and
// returns D(c[n]) ^ prev[n] in prev[n] (CBC, cyr_rijndael.cpp:625-630).
// A/B variant (r06), measured and not kept: the last
// round's 16 Si lookups per block from global memory (the TA path) instead of
// the LDS, so they would run beside the LDS gathers.  They do not: independent
// VMEM gathers from a small table sustain ~2.5 lookups / clk / CU against the
// LDS's ~27 (tools/microbench.hip k_vmix: 4 VMEM gathers per 16 LDS lookups
// cut the LDS rate from 26.6 to 10.1 per clk), and the decrypt needs ~3 Si
// lookups / clk / CU: config C decrypt 11.12 -> 13.38 ms, config B 1.024 ->
// 1.264 ms, bit-exact (profiles/r06/vmem/).
#ifndef CYAES_DEC_SI_VMEM
#define CYAES_DEC_SI_VMEM 0
#endif
// The inverse S-box bytes in global memory (kSiOff), from a decrypt's table pointer (kDecTableOff).
__device__ __forceinline__ const uint8_t* si_bytes(const uint32_t* dec_tables) {
    return reinterpret_cast<const uint8_t*>(dec_tables) + (kSiOff - kDecTableOff);
}
// Last-round word from global memory: Si[byte k of x_k] in byte k (the LDS
// form is dec_last).  global_load_ubyte gathers from one 256-B table: two
// 128-B lines, L1 resident; served by the TA path beside the LDS.
__device__ __forceinline__ uint32_t dec_last_g(const uint8_t* __restrict__ si, uint32_t x0, uint32_t x1, uint32_t x2,
                                               uint32_t x3) {
    const uint32_t l0 = si[x0 & 0xFFu], l1 = si[(x1 >> 8) & 0xFFu], l2 = si[(x2 >> 16) & 0xFFu], l3 = si[x3 >> 24];
    return l0 | (l1 << 8) | (l2 << 16) | (l3 << 24);
}

template <int N>
__device__ __forceinline__ void dec_cbc(const char* lds, uint32_t lo, const uint32_t* __restrict__ dk,
                                        const uint4 (&c)[N], uint4 (&prev)[N], const uint8_t* __restrict__ gsi = nullptr) {
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
#if CYAES_DEC_SI_VMEM
    if (gsi) {
#pragma unroll
        for (int n = 0; n < N; n++)
            prev[n] = make_uint4(xor3(dec_last_g(gsi, s[n][0], s[n][3], s[n][2], s[n][1]), dk[40], prev[n].x),
                                 xor3(dec_last_g(gsi, s[n][1], s[n][0], s[n][3], s[n][2]), dk[41], prev[n].y),
                                 xor3(dec_last_g(gsi, s[n][2], s[n][1], s[n][0], s[n][3]), dk[42], prev[n].z),
                                 xor3(dec_last_g(gsi, s[n][3], s[n][2], s[n][1], s[n][0]), dk[43], prev[n].w));
        return;
    }
#endif
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
#ifndef CYAES_ENC_PRIO_DIV
#define CYAES_ENC_PRIO_DIV 1
#endif
#ifndef CYAES_DEC_PRIO_DIV
#define CYAES_DEC_PRIO_DIV 8
#endif
// steps = 8-block chunks.  r01 A/B on config C: 1, 2, 4, 8 -> 4 best; r03 (after the
// runs and the coalesced moves): 1 -> configs B / D / relay stream -4.5 to -4.8 %
// (their ~1 ms launches end with a 12 % wave spread at 4), config C unchanged
// (profiles/r03/ab_prio_div_s2.txt).
constexpr uint32_t kEncPrioDiv = CYAES_ENC_PRIO_DIV;
constexpr uint32_t kDecPrioDiv = CYAES_DEC_PRIO_DIV;  // steps = 64*kDecRows-block rows (r01 A/B: 4, 8, 16 -> 8)
// Launches with few steps per wave (the MTU configs, relay streams: ~92) level
// their waves better at 4 (r04, static split: config B decrypt -2.8 %, the
// strided relay stream -4.7 %; config C +0.5 % at 4, so it keeps 8:
// profiles/r04/ab_dec_prio_div.txt).
#ifndef CYAES_DEC_PRIO_DIV_SHORT
#define CYAES_DEC_PRIO_DIV_SHORT 4
#endif
constexpr uint32_t kDecPrioDivShort = CYAES_DEC_PRIO_DIV_SHORT;

__device__ __forceinline__ uint4 default_iv() { return make_uint4(kIv0, kIv1, kIv2, kIv3); }

#if CYAES_CLOCK_PROBE
// Variant builds only (make probe): per-wave shader cycles (s_memtime) and
// wall ticks (s_memrealtime, 100 MHz per tools/clockcal.hip) over the kernel
// body, summed per kernel kind into g_probe and read by cyaes_debug_probe()
// (bench.py and tools/ab.py print the clock).
__device__ unsigned long long g_probe[2][4];  // [enc, dec] x {cycles, ticks, waves, max ticks}
// Per-wave timeline of the last launch of each kind (tools/timeline.py): wave
// slot blockIdx.x * waves per block + wave: {start ticks, end ticks (low 32
// bits of s_memrealtime), HW_ID, XCC_ID}, {cycles (s_memtime) low, high,
// blockIdx.x, wave in block}.
constexpr uint32_t kTimelineWaves = 8192;
__device__ uint4 g_timeline[2][kTimelineWaves][2];
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
            const uint32_t w = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
            if (w < kTimelineWaves) {
                const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID
                const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // HW_REG_XCC_ID
                g_timeline[kind][w][0] = make_uint4((uint32_t)r0, (uint32_t)r1, hw, xcc);
                g_timeline[kind][w][1] = make_uint4((uint32_t)(t1 - t0), (uint32_t)((t1 - t0) >> 32), blockIdx.x,
                                                    threadIdx.x >> 6);
            }
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

// v (lane l-1) for lanes 1..63, old for lane 0: DPP wave_shr:1.
__device__ __forceinline__ uint32_t shr1(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint4 shr1(uint4 v, uint4 old) {
    return make_uint4(shr1(v.x, old.x), shr1(v.y, old.y), shr1(v.z, old.z), shr1(v.w, old.w));
}

// Host readers of this TU's debug records (variant builds).
#if CYAES_BOUNDS_CHECK
inline int read_bounds_local(unsigned long long* rec4, unsigned int* lines) {
    if (hipMemcpyFromSymbol(rec4, HIP_SYMBOL(g_bounds), sizeof(unsigned long long) * 4) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(lines, HIP_SYMBOL(g_bounds_lines), sizeof(unsigned int) * kBoundsLines) != hipSuccess)
        return -1;
    static const unsigned long long zero[4] = {};
    static const unsigned int zl[kBoundsLines] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_bounds_lines), zl, sizeof(zl)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_bounds), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif
#if CYAES_CLOCK_PROBE
inline int read_timeline_local(int kind, uint4* out) {  // kTimelineWaves x 2 records, then cleared
    const size_t bytes = sizeof(uint4) * 2 * kTimelineWaves;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_timeline), bytes, bytes * kind) != hipSuccess) return -1;
    static uint4 zero[2 * kTimelineWaves];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_timeline), zero, bytes, bytes * kind) == hipSuccess ? 0 : -1;
}
inline int read_probe_local(unsigned long long* out8) {
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_probe), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    static const unsigned long long zero[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_probe), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace
}  // namespace cyaes
