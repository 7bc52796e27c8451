// cyaes_lines_body.h -- relay streams (strided batches) encrypted from 64-B
// lines: the walk of k_encrypt_lines (cyaes_enc_kernels.hip), one lane per
// payload chain (cyr_rijndael.cpp:588-609).  TU-local.
//
// A relay packet's payload sits at packet offset 12 (relay_server.cpp:329,
// relay_local.cpp:206), so on a stream of 1,484-B packets every payload starts
// 4-B aligned at a different phase of the 64-B line.  Coalesced 64-B loads
// at such positions move each group's bytes across two lines: that alone cost
// the relay stream's encrypt +7 % against the same loads from line starts
// (cost probe, profiles/r05/probe_align.txt; misaligned stores cost nothing,
// and rounding the loads to 16 B bought nothing).  Here a lane's work item is
// read as the aligned 64-B lines that hold its payload, two lines (a "chunk")
// per step, and the blocks are cut out of the lines in registers:
//  * wave g takes payloads 1024 (g / 16) + g % 16 + 16 l (l = lane), so
//    16 * stride == 0 mod 64 gives every payload of the wave the same line
//    phase m: the cut (below) is wave-uniform, and the group k, k+16, k+32,
//    k+48 (payloads 256 apart) loads one line of one payload per instruction;
//    transpose4 then gives each lane its own payload's blocks;
//  * with s = m / 4 the payload's dword i is dword i + s of the line stream;
//    chunk t holds dwords [32t, 32t + 32) and processes the blocks that END in
//    it, so slot j of chunk t (block 8t - j0 + j, j0 = (s + 3) / 4) is dwords
//    e + 4j .. e + 4j + 3 of W = {the last 3 dwords of chunk t-1, the chunk's
//    32}, e = (s + 3) % 4: one wave-uniform cut (32 register moves) per chunk.
//    (Folding the cut into per-slot variants of the first xor3 instead, with no
//    moves, split every slot's rounds into their own schedule region: +58 %,
//    profiles/r05/ab_enc_lines.txt);
//  * the next item's first chunk is loaded during the current item's last, so
//    only a wave's first item starts on an exposed load;
//  * stores stay the coalesced 64-B runs at the payload's own positions.
// Reads stay inside the lines that hold payload bytes (no page is touched that
// the payload does not touch); in place, each byte is read before its block is
// written (a chunk's stores end in its own lines; the next chunk's loads, of
// the lines after them, are issued before them).  A launch covers whole
// 1,024-payload groups (the runtime runs the rest through the other kernels);
// unkeyed, no IV arrays; offsets from the stream base are 32-bit (the runtime
// checks the span).
#pragma once

#include "cyaes_enc_body.h"

namespace cyaes {
namespace {

#ifndef CYAES_PROBE_LINES
#define CYAES_PROBE_LINES 0  // cost probes only (wrong output): bit 1 stores at 16-B aligned positions
#endif
#ifndef CYAES_RAG_MPOS_LDS
#define CYAES_RAG_MPOS_LDS 1  // 0: A/B variant, rag_lines_walk's member positions by four shuffles
#endif
#ifndef CYAES_RAG_BN_ZERO
#define CYAES_RAG_BN_ZERO 1  // 0: A/B variant, the next-chunk registers undefined on an item's last chunk
#endif
#ifndef CYAES_RAG_META_PF
#define CYAES_RAG_META_PF 1  // 0: A/B variant, rag_lines_walk loads an item's offsets and sizes at its start
#endif
#ifndef CYAES_LINES_PF
#define CYAES_LINES_PF 1  // 0: A/B variant without the next item's prefetch
#endif

// Dword k (-3 <= k < 32) of W: the carry for k < 0, else dword k of the chunk.
__device__ __forceinline__ uint32_t wdw_rt(const uint4 (&b)[8], uint32_t c0, uint32_t c1, uint32_t c2, int k) {
    if (k < 0) return k == -3 ? c0 : k == -2 ? c1 : c2;
    const uint4& v = b[k >> 2];
    return (k & 3) == 0 ? v.x : (k & 3) == 1 ? v.y : (k & 3) == 2 ? v.z : v.w;
}

// The walk, after the encrypt image is in LDS and *lead (LDS) is zero.  Row 0
// of the key table; every payload is its own chain from DefaultIV (the relay
// passes iv = nullptr).  The kernel arguments are read where used (passed in
// as values, they stayed live in SGPRs and the spills cost VGPRs: 128 with 7
// spilled, against 122).
__device__ __forceinline__ void lines_walk(const EncArgs& a, const char* lds, uint32_t* lead) {
    uint32_t prog = 0;
    const uint32_t pb = a.payload_bytes;
    const uint32_t lo = ((threadIdx.x & 31u) << 2) | 0x10000u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t mem = lane >> 4;
    const uint32_t nb = pb >> 4;
    // the loads and stores take a scalar base per group member (the members'
    // payloads are tstr apart) and one lane offset per chunk
    const uint32_t tstr = 256u * (uint32_t)a.stride;
    uint32_t ek[44];
    load_sched(a.keys, 0, 0, ek);
    // Global wave gw takes phase gw % 16 of payload group gw / 16 (any block size)
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * wpb, gwaves = a.npayloads / 64u;
    // A work item's placement: the group's payload offset (VGPR), its line
    // phase and what follows from it (wave-uniform).
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
        const uint64_t gwn = gw + nwaves;
        const bool has_next = CYAES_LINES_PF && gwn < gwaves;
        const Item nx = has_next ? item_of(gwn) : it;
        const uint32_t goff = it.goff, e = it.e, j0 = it.j0, nchunks = it.nchunks;
        uint32_t c0 = 0, c1 = 0, c2 = 0;  // the last 3 dwords of the previous chunk
        uint4 c = default_iv();
        for (uint32_t t = 0; t < nchunks; t++) {
            const bool more = t + 1 < nchunks;
            const uint32_t jlo = t == 0 ? j0 : 0u;
            const uint32_t jhi = min(8u, nb + j0 - 8u * t);
            // The cut: one uniform branch per chunk, then each slot's 4 dwords are moves.
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
            // the next chunk's loads, in flight during this one's rounds (after the
            // cut, so b and the loads' registers are not live together)
            uint4 bn[8];
            if (more) load_chunk(it, bn, t + 1);
            else if (has_next) load_chunk(nx, bn, 0);
            prio_feedback(lead, ++prog, kEncPrioDiv);
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

// Ragged (list) batches by lines (r06): k_encrypt_lines
// over the first whole 1,024-payload groups of an unkeyed ragged batch without
// IV arrays.  Wave g takes the payloads lines_walk gives it (16 apart: a relay
// stream's waves are then phase-uniform whatever its packet size), loads its
// 64 offsets and sizes, and walks them exactly as lines_walk does when they
// share one line phase and one length and lie within 4 GiB - 64 B of the
// lowest of them, with the group members' positions (VGPRs, 32-bit) in place of
// the stride.  Any other wave appends its index to a.rest (count at [0]) and
// leaves its payloads to the ragged lane kernel, which walks that list next
// (enc_body, a.rest).  No prefetch of the next item's first chunk (the
// members' positions of two items at once did not fit the registers).
__device__ __forceinline__ void rag_lines_walk(const EncArgs& a, const char* lds, uint32_t* lead, uint32_t* mpos) {
    uint32_t prog = 0;
    const uint32_t lo = ((threadIdx.x & 31u) << 2) | 0x10000u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t mem = lane >> 4;
    uint32_t ek[44];
    load_sched(a.keys, 0, 0, ek);
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * wpb, gwaves = a.npayloads / 64u;
    const uintptr_t in0 = reinterpret_cast<uintptr_t>(a.in);
    auto pl_of = [&](uint64_t g) { return (g >> 4) * 1024u + (g & 15u) + 16u * lane; };  // this lane's payload
#if CYAES_RAG_META_PF
    // the next item's offsets and sizes load during this item's chunks
    uint64_t g = (uint64_t)blockIdx.x * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t off_n = 0;
    uint32_t nbr_n = 0;
    if (g < gwaves) {
        off_n = LD8(a.offsets + pl_of(g), ext(a.offsets, 8 * a.npayloads));
        nbr_n = LD4(a.nbytes + pl_of(g), ext(a.nbytes, 4 * a.npayloads));
    }
    for (; g < gwaves; g += nwaves) {
        const uint64_t off = off_n;
        const uint32_t nb = nbr_n >> 4;
        if (g + nwaves < gwaves) {
            off_n = LD8(a.offsets + pl_of(g + nwaves), ext(a.offsets, 8 * a.npayloads));
            nbr_n = LD4(a.nbytes + pl_of(g + nwaves), ext(a.nbytes, 4 * a.npayloads));
        }
#else
    for (uint64_t g = (uint64_t)blockIdx.x * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); g < gwaves;
         g += nwaves) {
        const uint64_t off = LD8(a.offsets + pl_of(g), ext(a.offsets, 8 * a.npayloads));
        const uint32_t nb = LD4(a.nbytes + pl_of(g), ext(a.nbytes, 4 * a.npayloads)) >> 4;
#endif
        const uint32_t nb0 = __builtin_amdgcn_readfirstlane(nb);
        const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(in0 + off) & 63u);
        uint64_t wlo = off;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t o2 = (uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(wlo >> 32), d) << 32 |
                                (uint32_t)__shfl_xor((int)(uint32_t)wlo, d);
            wlo = min(wlo, o2);
        }
        wlo = (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(wlo >> 32)) << 32 |
              __builtin_amdgcn_readfirstlane((uint32_t)wlo);
        const bool ok = nb0 > 0 && __ballot(nb != nb0 || ((uint32_t)(in0 + off) & 63u) != m ||
                                            off - wlo + 16ull * nb0 + 128u >= (1ull << 32)) == 0;
        if (!ok) {  // to the lane kernel
            if (lane == 0) {
                const uint32_t i = atomicAdd(a.rest, 1u);
                a.rest[1 + i] = (uint32_t)g;
            }
            continue;
        }
        // base: the lowest payload's first line (may precede a.in by < 64 B, inside its line)
        const uint8_t* base = a.in + (wlo - m);
        uint8_t* obase = a.out + (wlo - m);
        // the group members' payloads (lanes k + 16 q): their first lines from
        // base, through the wave's 256 B of LDS (one address and immediate
        // offsets; lane-index registers for four shuffles were hoisted out of
        // the walk and spilled)
        uint32_t mrel[4];
#if CYAES_RAG_MPOS_LDS
        uint32_t* wpos = mpos + (threadIdx.x & ~63u);
        wpos[lane] = (uint32_t)(off - wlo);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 4; q++) mrel[q] = wpos[(lane & 15u) + 16u * q];
        __builtin_amdgcn_wave_barrier();
#else
#pragma unroll
        for (int q = 0; q < 4; q++) mrel[q] = (uint32_t)__shfl((int)(uint32_t)(off - wlo), (int)((lane & 15u) + 16u * q));
#endif
        const uint32_t s = m >> 2;
        const uint32_t e = (s + 3u) & 3u, j0 = (s + 3u) >> 2;
        const uint32_t nlines = (m + 16u * nb0 + 63u) >> 6;
        const uint32_t nchunks = (nb0 - 1u + j0) / 8u + 1u;
        auto load_chunk = [&](uint4 (&v)[8], uint32_t t) {
            const uint32_t l1 = min(2u * t + 1u, nlines - 1u) - 2u * t;  // 1, or 0 past the last line
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t lo64 = (j >> 2) ? 64u * l1 : 0u;
                v[j] = LD16(base + (mrel[j & 3] + 128u * t + lo64 + 16u * mem), ext(base + mrel[j & 3], 64ull * nlines));
            }
        };
        uint4 b[8];
        load_chunk(b, 0);
        transpose4(b), transpose4(b + 4);
        uint32_t c0 = 0, c1 = 0, c2 = 0;
        uint4 c = default_iv();
        for (uint32_t t = 0; t < nchunks; t++) {
            const bool more = t + 1 < nchunks;
            const uint32_t jlo = t == 0 ? j0 : 0u;
            const uint32_t jhi = min(8u, nb0 + j0 - 8u * t);
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
            uint4 bn[8];
            if (more) {
                load_chunk(bn, t + 1);
            } else if (CYAES_RAG_BN_ZERO) {
                // defined on the last chunk: left undefined, the registers were
                // carried (and spilled, 22 VGPRs) from item to item
#pragma unroll
                for (int j = 0; j < 8; j++) bn[j] = make_uint4(0u, 0u, 0u, 0u);
            }
            prio_feedback(lead, ++prog, kEncPrioDiv);
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
            transpose4(o), transpose4(o + 4);
            const uint32_t soff = m + 16u * (8u * t - j0 + mem);  // (32-bit: wraps below 0 before j0 in chunk 0)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t sl = mem + 4u * (uint32_t)(j >> 2);
                if (sl >= jlo && sl < jhi)
                    ST16U(obase + (mrel[j & 3] + soff + 64u * (uint32_t)(j >> 2)),
                          ext(obase + mrel[j & 3] + m, 16ull * nb0), o[j]);
            }
            if (more) {
#pragma unroll
                for (int j = 0; j < 8; j++) b[j] = bn[j];
                transpose4(b), transpose4(b + 4);
            }
        }
    }
}

}  // namespace
}  // namespace cyaes
