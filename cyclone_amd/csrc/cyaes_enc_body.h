// cyaes_enc_body.h -- the CBC encrypt walk of k_encrypt (one lane per payload
// chain, cyr_rijndael.cpp:588-609 + _encryptBlock :638-705), shared by the
// encrypt translation unit (cyaes_enc_kernels.hip) and the duplex kernel
// (cyaes_duplex_kernels.hip).  Included after cyaes_device.h; TU-local.
#pragma once

#include <type_traits>

#include "cyaes_device.h"

namespace cyaes {
namespace {

#ifndef CYAES_ENC_COAL
#define CYAES_ENC_COAL 1
#endif
#ifndef CYAES_ENC_COAL_RAGGED
#define CYAES_ENC_COAL_RAGGED 1
#endif
// Cost probe builds only (wrong output): coalesced ragged loads (bit 0) and/or
// stores (bit 1) from the work item's offset rounded down to 64 B (bit 2: loads
// rounded down to 16 B), to price
// the payloads' 4-B alignment on relay streams.
#ifndef CYAES_PROBE_RAGGED_ALIGN
#define CYAES_PROBE_RAGGED_ALIGN 0
#endif

// 4x4 transpose of 16-B blocks among the lanes k, k+16, k+32, k+48 (rows of
// the wave, "members" m = lane >> 4): member m's r[t] becomes member t's r[m].
// Two butterfly stages, one v_permlane16_swap / v_permlane32_swap per dword
// and register pair (gfx950), in place.
__device__ __forceinline__ void swap16(uint32_t& x, uint32_t& y) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    x = r[0];
    y = r[1];
}
__device__ __forceinline__ void swap32(uint32_t& x, uint32_t& y) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    x = r[0];
    y = r[1];
}
__device__ __forceinline__ void swap16(uint4& a, uint4& b) {
    swap16(a.x, b.x), swap16(a.y, b.y), swap16(a.z, b.z), swap16(a.w, b.w);
}
__device__ __forceinline__ void swap32(uint4& a, uint4& b) {
    swap32(a.x, b.x), swap32(a.y, b.y), swap32(a.z, b.z), swap32(a.w, b.w);
}
__device__ __forceinline__ void transpose4(uint4* r) {
    swap16(r[0], r[1]);
    swap16(r[2], r[3]);
    swap32(r[0], r[2]);
    swap32(r[1], r[3]);
}

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
// Fills the 128 KiB encrypt image (the first 32,768 words of lds_words).
__device__ __forceinline__ void fill_enc_image(uint32_t* lds_words, const uint32_t* tables) {
    fill_region(lds_words, tables, tables + 512, blockDim.x);              // TL1 | TL3
    fill_region(lds_words + 16384, tables + 256, tables + 768, blockDim.x);  // TL2 | TL4
}

// The walk itself, after the image is in LDS and the workgroup's
// progress-feedback word (*lead, LDS) is zero.
template <bool RAGGED, bool KEYED, bool RUNS, bool SESS>
__device__ __forceinline__ void enc_body(const EncArgs& a, const char* lds, uint32_t* lead) {
    uint32_t prog = 0;
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
        if (RAGGED && a.stride) {  // strided batch: the positions are arithmetic
            off = active ? a.off0 + p * a.stride : 0;
            nb = active ? bpp : 0;
        } else if (RAGGED) {
            off = active ? LD8(a.offsets + p, ext(a.offsets, 8 * a.npayloads)) : 0;
            nb = active ? (LD4(a.nbytes + p, ext(a.nbytes, 4 * a.npayloads)) >> 4) : 0;
        } else {
            off = p * (uint64_t)a.payload_bytes;
            nb = active ? (RUNS ? (uint32_t)min<uint64_t>(R, a.npayloads - p) * bpp : bpp) : 0;
        }
        // RUNS + KEYED: the runtime makes runs divide payloads_per_key, so the run is one session
        const uint32_t kid = KEYED ? key_index(a.keys, p, a.npayloads, active, a.status) : 0u;
        // Coalesced chunk moves (batches without per-lane keys or IV arrays, full
        // waves of equal work items; ragged batches only in place): load / store j
        // of a chunk moves 64 contiguous bytes of one work item with the 4 lanes
        // k, k+16, k+32, k+48, and the blocks reach their own lanes by transpose4.
        // A wave instruction then touches 16 half-lines instead of 64 lines, which
        // the power-limited clock repays (config C encrypt -2 %), and a relay
        // stream's misaligned payloads are stored 64 contiguous bytes at a time
        // (1 M relay packets in place -6 %; out of place it measured +3 %, so
        // out-of-place ragged batches keep the per-lane moves;
        // profiles/r03/ab_enc_coalesced.txt).
        const bool coal = CYAES_ENC_COAL && (!RAGGED || (CYAES_ENC_COAL_RAGGED && a.in == a.out)) && !KEYED &&
                          a.iv_in == nullptr && __ballot(active && nb == __builtin_amdgcn_readfirstlane(nb)) == ~0ull;
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
                // coal: member 0's work item of this lane's group, and the bytes between members
                const uint32_t mem = lane >> 4;
                const uint64_t mstride = 16ull * R * a.payload_bytes;
                const uint8_t* gsrc = src - mem * mstride;
                uint8_t* gdst = dst - mem * mstride;
                const Ext ge = ext(a.in, (uint64_t)a.npayloads * a.payload_bytes);
                const Ext gde = ext(a.out, (uint64_t)a.npayloads * a.payload_bytes);
                uint64_t moff[4] = {0, 0, 0, 0};  // ragged coal: byte offsets of the group's work items
                if constexpr (RAGGED) {
                    if (coal) {
#pragma unroll
                        for (int t = 0; t < 4; t++) {
                            const int from = (int)((lane & 15u) + 16u * t);
                            moff[t] = (uint64_t)(uint32_t)__shfl((int)(uint32_t)(off >> 32), from) << 32 |
                                      (uint32_t)__shfl((int)(uint32_t)off, from);
                        }
                    }
                }
                // 8 blocks from block kk of this lane's work item into v[0..7]; coal:
                // still transposed (the caller transposes once the loads have landed,
                // so a prefetch stays in flight during the chunk's rounds)
                auto load8 = [&](auto co_tag, uint4 (&v)[8], uint32_t kk) {
                    if constexpr (decltype(co_tag)::value && RAGGED) {
#pragma unroll
                        for (int j = 0; j < 8; j++) {
                            const uint8_t* w0 = a.in + (moff[j & 3] & ((CYAES_PROBE_RAGGED_ALIGN & 1) ? ~63ull : (CYAES_PROBE_RAGGED_ALIGN & 4) ? ~15ull : ~0ull));
                            v[j] = LD16U(w0 + 16ull * (kk + 4 * (j >> 2) + mem), ext(w0, 16ull * nb));
                        }
                    } else if constexpr (decltype(co_tag)::value) {
                        const uint8_t* q = gsrc + 16ull * (kk + mem);
#pragma unroll
                        for (int j = 0; j < 8; j++) v[j] = LD16(q + (j & 3) * mstride + 64 * (j >> 2), ge);
                    } else {
                        const uint8_t* q = src + 16ull * kk;
#pragma unroll
                        for (int j = 0; j < 8; j++) v[j] = ldb<RAGGED>(q, j, se);
                    }
                };
                // The chunk loop, with the coalesced moves compiled in or out (one
                // branch per work item: inside the loop a join of the two store paths
                // made the compiler drain every store before the next loads).
                auto chunks = [&](auto co_tag) {
                    constexpr bool CO = decltype(co_tag)::value;
                    uint4 b[8];
                    if (nb >= 8) {
                        load8(co_tag, b, 0);
                        if constexpr (CO) transpose4(b), transpose4(b + 4);
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
                        if (more || tail) load8(co_tag, bn, more ? i + 8 : nb - 8);
                        prio_feedback(lead, ++prog, kEncPrioDiv);
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
                        if constexpr (CO) {  // the transposes back, then 64 contiguous bytes of one work item per store
                            transpose4(b);
                            transpose4(b + 4);
                            if constexpr (RAGGED) {
#pragma unroll
                                for (int j = 0; j < 8; j++) {
                                    uint8_t* w0 = a.out + (moff[j & 3] & ((CYAES_PROBE_RAGGED_ALIGN & 2) ? ~63ull : ~0ull));
                                    ST16U(w0 + 16ull * (i + 4 * (j >> 2) + mem), ext(w0, 16ull * nb), b[j]);
                                }
                            } else {
                                uint8_t* const q = gdst + 16ull * (i + mem);
#pragma unroll
                                for (int j = 0; j < 8; j++) ST16(q + (j & 3) * mstride + 64 * (j >> 2), gde, b[j]);
                            }
                        } else {
                            uint8_t* const dchunk = dst + 16ull * i;  // one address, immediate offsets (ragged too)
#pragma unroll
                            for (int j = 0; j < 8; j++) stb<RAGGED>(dchunk, j, b[j], de);  // (nt stores measured 3.6x slower)
                        }
                        if (more || tail) {
#pragma unroll
                            for (int j = 0; j < 8; j++) b[j] = bn[j];
                            if constexpr (CO) transpose4(b), transpose4(b + 4);
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
                };
                if constexpr (!KEYED && (!RAGGED || CYAES_ENC_COAL_RAGGED)) {
                    if (coal) chunks(std::true_type{});
                    else chunks(std::false_type{});
                } else {
                    chunks(std::false_type{});
                }
                if (a.iv_out) ST16(a.iv_out + 16 * p, iv_out_e, c);  // (RUNS: no IV arrays)
            }
        }
        if (SESS) break;  // one pass (above)
    }
}

// ---- Strided batches read by 64-B lines (relay streams, k_encrypt_lines) ----
// A relay packet's payload sits at packet offset 12 (relay_server.cpp:329,
// relay_local.cpp:206), so on a stream of 1,484-B packets every payload starts
// 4-B aligned at a different phase of the 64-B line.  The coalesced loads of
// enc_body then move each group's 64 bytes across two lines: that alone costs
// the relay stream's encrypt +7 % against the same loads from line starts
// (cost probe, profiles/r05/probe_align.txt; the misaligned stores cost
// nothing).  Here a lane's work item is read as the aligned 64-B lines that
// hold its payload, two lines (a "chunk") per step, and the blocks are cut out
// of the lines in registers:
//  * wave g takes payloads 1024 (g / 16) + g % 16 + 16 l (l = lane), so
//    16 * stride == 0 mod 64 gives every payload of the wave the same
//    line phase m: the cut (below) is wave-uniform, and the group k, k+16,
//    k+32, k+48 (payloads 256 apart) still loads one line of one payload per
//    instruction;
//  * with s = m / 4 the payload's dword i is dword i + s of the line stream;
//    chunk t holds dwords [32t, 32t + 32) and processes the blocks that END in
//    it, so slot j of chunk t (block 8t - j0 + j, j0 = (s + 3) / 4) is dwords
//    e + 4j .. e + 4j + 3 of W = {the last 3 dwords of chunk t-1, the chunk's
//    32}, e = (s + 3) % 4: one wave-uniform cut (32 register moves) per chunk;
//  * stores stay the coalesced 64-B runs at the payload's own positions.
// Reads stay inside the lines that hold payload bytes (no page is touched
// that the payload does not touch); in place, each byte is read before its
// block is written (a chunk's stores end in its own lines; the next chunk's
// loads start after them).  The launch covers whole 1,024-payload groups
// (the runtime runs the rest through enc_body); unkeyed, no IV arrays.
#ifndef CYAES_PROBE_LINES
#define CYAES_PROBE_LINES 0  // cost probes only (wrong output): bit 1 stores at 16-B aligned positions
#endif
// Dword k (-3 <= k < 32) of W: the carry for k < 0, else dword k of the chunk.
__device__ __forceinline__ uint32_t wdw_rt(const uint4 (&b)[8], uint32_t c0, uint32_t c1, uint32_t c2, int k) {
    if (k < 0) return k == -3 ? c0 : k == -2 ? c1 : c2;
    const uint4& v = b[k >> 2];
    return (k & 3) == 0 ? v.x : (k & 3) == 1 ? v.y : (k & 3) == 2 ? v.z : v.w;
}
#ifndef CYAES_LINES_PF
#define CYAES_LINES_PF 1  // 0: A/B variant without the next item's prefetch
#endif
__device__ __forceinline__ void enc_lines_body(const EncArgs& a, const char* lds, uint32_t* lead) {
    uint32_t prog = 0;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lo = ((threadIdx.x & 31u) << 2) | 0x10000u;
    const uint32_t mem = lane >> 4;
    const uint32_t pb = a.payload_bytes, nb = pb >> 4;
    // Offsets from the stream base are 32-bit (the runtime checks the span):
    // the loads and stores take a scalar base per group member (the members'
    // payloads are tstr apart) and one lane offset per chunk.
    const uint32_t tstr = 256u * (uint32_t)a.stride;
    uint32_t ek[44];
    load_sched(a.keys, 0, 0, ek);
    // Global wave gw takes phase gw % 16 of payload group gw / 16 (any block size)
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * wpb, gwaves = a.npayloads / 64u;
    // A work item's placement: the group's payload offset (VGPR) and its line
    // phase and the quantities derived from it (wave-uniform).
    struct Item {
        uint32_t goff, aloff, m, e, j0, nlines, nchunks;
    };
    auto item_of = [&](uint64_t g) {
        Item it;
        // member 0's payload of this lane's group; member t's is 256 t further
        const uint32_t pg = (uint32_t)(g >> 4) * 1024u + (uint32_t)(g & 15u) + 16u * (lane & 15u);
        it.goff = (uint32_t)a.off0 + pg * (uint32_t)a.stride;
        it.m = __builtin_amdgcn_readfirstlane(((uint32_t)reinterpret_cast<uintptr_t>(a.in) + it.goff) & 63u);
        it.aloff = it.goff - it.m + 16u * mem;  // this member's 16 B of the group's first line
        const uint32_t s = it.m >> 2;
        it.e = (s + 3u) & 3u;
        it.j0 = (s + 3u) >> 2;
        it.nlines = (it.m + pb + 63u) >> 6;
        it.nchunks = (nb - 1u + it.j0) / 8u + 1u;
        return it;
    };
    // The two lines of chunk t for the group's 4 payloads, still transposed.
    // A line past the payload's last (the last chunk's second, when the
    // payload ends in its first) re-reads the last one: unconditional loads,
    // so no wait is forced on the loads in flight.
    auto load_chunk = [&](const Item& it, uint4 (&v)[8], uint32_t t) {
        const uint32_t l1 = min(2u * t + 1u, it.nlines - 1u) - 2u * t;  // 1, or 0 past the end
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint8_t* sb = a.in + (uint32_t)(j & 3) * tstr;  // scalar
            const uint32_t lo64 = (j >> 2) ? 64u * l1 : 0u;
            v[j] = LD16(sb + (it.aloff + 128u * t + lo64), ext(sb + (it.goff - it.m), 64ull * it.nlines));
        }
    };
    uint64_t gw = (uint64_t)blockIdx.x * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (gw >= gwaves) return;
    Item it = item_of(gw);
    uint4 b[8];
    load_chunk(it, b, 0);
    transpose4(b), transpose4(b + 4);
    while (true) {
        // The next work item's first chunk is loaded during this one's last
        // chunk, so only the wave's first item starts on an exposed load.
        const uint64_t gwn = gw + nwaves;
        const bool has_next = CYAES_LINES_PF && gwn < gwaves;
        const Item nx = has_next ? item_of(gwn) : it;
        const uint32_t goff = it.goff, e = it.e, j0 = it.j0, nchunks = it.nchunks;
        uint32_t c0 = 0, c1 = 0, c2 = 0;  // the last 3 dwords of the previous chunk
        uint4 c = default_iv();
        for (uint32_t t = 0; t < nchunks; t++) {
            const bool more = t + 1 < nchunks;
            uint4 bn[8];
            if (more) load_chunk(it, bn, t + 1);
            else if (has_next) load_chunk(nx, bn, 0);
            prio_feedback(lead, ++prog, kEncPrioDiv);
            const uint32_t jlo = t == 0 ? j0 : 0u;
            const uint32_t jhi = min(8u, nb + j0 - 8u * t);
            // The cut: one uniform branch per chunk, then each slot's 4 dwords are moves
            // (folding the cut into per-slot variants of the first xor3 instead, with no
            // moves, split every slot's rounds into their own schedule region: +58 %).
            uint4 o[8];
            auto cut = [&](auto et) {
                constexpr int E = decltype(et)::value;
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const int K = E - 3 + 4 * j;
                    o[j] = make_uint4(wdw_rt(b, c0, c1, c2, K), wdw_rt(b, c0, c1, c2, K + 1),
                                      wdw_rt(b, c0, c1, c2, K + 2), wdw_rt(b, c0, c1, c2, K + 3));
                }
            };
            if (e == 3) cut(std::integral_constant<int, 3>{});
            else if (e == 2) cut(std::integral_constant<int, 2>{});
            else if (e == 1) cut(std::integral_constant<int, 1>{});
            else cut(std::integral_constant<int, 0>{});
            c0 = b[7].y, c1 = b[7].z, c2 = b[7].w;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if ((uint32_t)j >= jlo && (uint32_t)j < jhi) {
                    uint32_t s0 = xor3(c.x, o[j].x, ek[0]), s1 = xor3(c.y, o[j].y, ek[1]);
                    uint32_t s2 = xor3(c.z, o[j].z, ek[2]), s3 = xor3(c.w, o[j].w, ek[3]);
                    enc_block(lds, lo, ek, s0, s1, s2, s3);
                    c = make_uint4(s0, s1, s2, s3);
                    o[j] = c;
                }
            }
            // back to the group's payloads: member mem then holds slot mem + 4 (j >> 2) of payload j & 3
            transpose4(o), transpose4(o + 4);
            const uint32_t soff = goff + 16u * (8u * t - j0 + mem);  // slot mem's block (t == 0: slots >= j0 only)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t sl = mem + 4u * (uint32_t)(j >> 2);
                uint8_t* sb = a.out + (uint32_t)(j & 3) * tstr;  // scalar
                // (32-bit sum: soff wraps below 0 for the slots before j0 of chunk 0)
                if (sl >= jlo && sl < jhi)
                    ST16U(sb + ((soff + 64u * (uint32_t)(j >> 2)) & ((CYAES_PROBE_LINES & 2) ? ~15u : ~0u)),
                          ext(sb + goff, pb), o[j]);
            }
            if (more || has_next) {
#pragma unroll
                for (int j = 0; j < 8; j++) b[j] = bn[j];
                transpose4(b), transpose4(b + 4);
            }
        }
        if (!CYAES_LINES_PF) {  // (A/B variant: each item's first chunk loaded at its start)
            gw = gwn;
            if (gw >= gwaves) break;
            it = item_of(gw);
            load_chunk(it, b, 0);
            transpose4(b), transpose4(b + 4);
            continue;
        }
        if (!has_next) break;
        gw = gwn;
        it = nx;
    }
}


}  // namespace
}  // namespace cyaes
