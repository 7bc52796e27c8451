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
    // RAGGED with a.rest: the waves k_encrypt_rag_lines handed back (their
    // count at rest[0], written by it earlier on the stream), each the 64
    // payloads 16 apart of a 1,024-payload group that the line walk gives a wave.
    const bool listed = RAGGED && a.rest != nullptr;
    const uint64_t nwork = listed ? 64ull * __builtin_amdgcn_readfirstlane(LD4(a.rest, ext(a.rest, 4)))
                                  : RUNS ? (a.npayloads + R - 1) / R : a.npayloads;
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
        uint64_t w = wbase + lane;
        const bool active = w < nwork;
        if (listed) {
            const uint32_t gw = __builtin_amdgcn_readfirstlane(
                LD4(a.rest + 1 + (wbase >> 6), ext(a.rest, 4 + 4 * (nwork >> 6))));
            w = (uint64_t)(gw >> 4) * 1024u + (gw & 15u) + 16u * lane;
        }
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

}  // namespace
}  // namespace cyaes
