// cyaes_dec_body.h -- the flat CBC decrypt walk of k_decrypt_flat (one lane
// per block, cyr_rijndael.cpp:612-635 + _decryptBlock :708-774), shared by the
// decrypt translation unit (cyaes_dec_kernels.hip) and the duplex kernel
// (cyaes_duplex_kernels.hip).  Included after cyaes_device.h; TU-local.
#pragma once

#include "cyaes_device.h"

namespace cyaes {
namespace {

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

// STRIDED batches (a relay stream of equal packets resident in HBM): payload p
// lies at byte off0 + p * stride (4-B aligned), so block r of payload p is at
// off0 + p * stride + 16 r; the flat block order, chaining and rows are the
// same as a contiguous batch's, only the addresses differ.
__device__ __forceinline__ uint64_t soff(const DecArgs& a, uint64_t p, uint32_t r) {
    return a.off0 + p * a.stride + 16ull * r;
}
__device__ __forceinline__ uint64_t soff_g(const DecArgs& a, uint64_t g) {  // flat block g (partial steps only)
    const uint64_t p = g / a.bpp.d;
    return soff(a, p, (uint32_t)(g - p * a.bpp.d));
}
__device__ __forceinline__ Ext data_ext(const uint8_t* base, const DecArgs& a, bool strided) {
    return strided ? ext(base + a.off0, (a.npayloads - 1) * a.stride + 16ull * a.bpp.d) : ext(base, 16 * a.nblocks);
}
// Position r of row k's block in its payload in a STRIDED !BIG full step, and
// the row's byte offset o (from in + off0), from row 0's (rk[0], pk[0] = its
// offset): rows are 64 blocks apart and payloads >= 64 blocks (the runtime's
// condition for STRIDED), so each row wraps at most once, and each wrap skips
// the gap between payloads (stride - payload bytes).  Only row 0's position
// is carried across steps: two VGPRs, where tracking every row took eight and
// the step loop lost its schedule at the 128-VGPR limit.
__device__ __forceinline__ void srow_pos(uint32_t bpp, uint32_t gap, int k, const uint32_t (&rk)[kDecRows],
                                         const uint32_t (&pk)[kDecRows], uint32_t& r, uint32_t& o) {
    r = rk[0];
    o = pk[0] + 1024u * k;
    for (int j = 0; j < k; j++) {
        const uint32_t t = r + 64;
        const bool wrap = t >= bpp;
        r = wrap ? t - bpp : t;
        o += wrap ? gap : 0u;
    }
}
// Byte offset (from in + off0) of row k's block in a STRIDED full step: !BIG
// from row 0's tracked offset, BIG from the step position (at most one payload
// start).  32-bit: the runtime runs this kernel only on streams that span less
// than 4 GiB, so the loads and stores take the scalar base + 32-bit lane
// offset form.  (With 64-bit per-row address arithmetic on both the loads and
// the stores, the step lost its schedule: 315 s_waitcnt per 640 LDS reads
// against 53.)
template <bool BIG>
__device__ __forceinline__ uint32_t srow(const DecArgs& a, FlatPos ps, uint32_t lane, int k, const uint32_t (&rk)[kDecRows],
                                         const uint32_t (&pk)[kDecRows]) {
    const uint32_t stride = (uint32_t)a.stride;
    if (BIG) {
        const uint32_t lpos = ps.bpos + 64 * k + lane;
        const bool next = lpos >= a.bpp.d;
        return (uint32_t)ps.bp * stride + (next ? stride - 16u * a.bpp.d : 0u) + 16u * lpos;
    }
    uint32_t r, o;
    srow_pos(a.bpp.d, stride - 16u * a.bpp.d, k, rk, pk, r, o);
    return o;
}

// Cost probe (CYAES_PROBE_DEC_ALIGN bit 1: loads, bit 2: stores; wrong
// output): the row's accesses moved to one contiguous 1-KiB run from lane
// 0's address rounded down to 64 B, i.e. what line-aligned rows would cost.
#ifndef CYAES_PROBE_DEC_ALIGN
#define CYAES_PROBE_DEC_ALIGN 0
#endif
template <int BIT, typename P>
__device__ __forceinline__ P* probe_dec_addr(P* base, uint32_t o, uint32_t lane) {
    if (!(CYAES_PROBE_DEC_ALIGN & BIT)) return base + o;
    const uint64_t r0 = reinterpret_cast<uint64_t>(base + __builtin_amdgcn_readfirstlane(o)) & ~63ull;
    return reinterpret_cast<P*>(r0 + 16ull * lane);
}

// Loads the R rows of the step at `base` (c); partial steps also load each
// block's predecessor (pv), full steps take it from the neighbour lane.
// FULL: all 64*R blocks are in range (every step but possibly the batch's
// last), so loads are unguarded and use immediate offsets off one lane pointer
// (STRIDED: one address per row).
template <bool FULL, bool BIG, bool STRIDED>
__device__ __forceinline__ void flat_load(const DecArgs& a, const uint8_t* in_s, uint32_t lane, uint64_t base,
                                          uint64_t end, FlatPos ps, const uint32_t (&rk)[kDecRows],
                                          const uint32_t (&pk)[kDecRows], uint4 (&c)[kDecRows], uint4 (&pv)[kDecRows]) {
    constexpr int R = kDecRows;
    const Ext ie = data_ext(a.in, a, STRIDED);
    if (FULL && STRIDED) {  // in_s = in + off0
#pragma unroll
        for (int k = 0; k < R; k++) c[k] = LD16U(probe_dec_addr<1>(in_s, srow<BIG>(a, ps, lane, k, rk, pk), lane), ie);
    } else if (FULL) {
        const uint8_t* g0 = a.in + 16 * (base + lane);
#pragma unroll
        for (int k = 0; k < R; k++) c[k] = LD16(g0 + 1024 * k, ie);
        // pv comes from the neighbour lane in flat_step (DPP), not from memory
    } else {  // last, partial step of the batch: clamp reads into range
#pragma unroll
        for (int k = 0; k < R; k++) {
            const uint64_t g = min(base + 64 * k + lane, end - 1);
            // The predecessor of block g (lane 0 of row 0 reads its own block:
            // the carry replaces it).  Block 0 has none: a 1-block batch (end
            // == 1) clamps every lane to g = 0, and g - 1 would read 16 B before
            // the buffer (r02 fault hunt, VERDICT r02 "What's weak" 1).  Block
            // 0 is a payload start, so its pv is the IV in flat_step anyway.
            const uint64_t back = (k == 0 && lane == 0) ? 0u : 1u;
            const uint64_t gp = g >= back ? g - back : 0u;
            if (STRIDED) {
                c[k] = LD16U(a.in + soff_g(a, g), ie);
                pv[k] = LD16U(a.in + soff_g(a, gp), ie);
            } else {
                c[k] = LD16(a.in + 16 * g, ie);
                pv[k] = LD16(a.in + 16 * gp, ie);
            }
        }
    }
}

template <bool KEYED, bool BIG, bool FULL, bool IV, bool STRIDED>
__device__ __forceinline__ uint4 flat_step(const DecArgs& a, const char* lds, uint32_t lo, uint32_t lane,
                                           uint64_t base, uint64_t end, FlatPos ps, uint4 carry,
                                           uint32_t (&dk0)[44], uint32_t& dk_id, const uint4 (&c)[kDecRows],
                                           uint4 (&pv)[kDecRows], const uint32_t (&rk)[kDecRows],
                                           const uint32_t (&pk)[kDecRows], uint8_t* out_s) {
    constexpr int R = kDecRows;
    const Ext oe = data_ext(a.out, a, STRIDED);
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
            const uint4 ivv = (IV && a.iv_in) ? LD16(a.iv_in + 16 * pf, iv_in_e) : default_iv();
#pragma unroll
            for (int k = 0; k < R; k++)
                if ((fo >> 6) == (uint32_t)k && lane == (fo & 63u)) pv[k] = ivv;
        }
    } else if (!IV || !a.iv_in) {  // chains restart at DefaultIV: a select on the lane's tracked position
#pragma unroll
        for (int k = 0; k < R; k++) {
            uint32_t r = rk[k], o;
            if (STRIDED) srow_pos(a.bpp.d, 0u, k, rk, pk, r, o);
            if (r == 0) pv[k] = default_iv();
        }
    } else {
#pragma unroll
        for (int k = 0; k < R; k++) {
            uint32_t r;
            uint64_t p;
            flat_position<BIG>(a, ps, lane, k, r, p);
            if (r == 0) {
                const bool valid = FULL || base + 64 * k + lane < end;
                pv[k] = valid ? LD16(a.iv_in + 16 * p, iv_in_e) : default_iv();
            }
        }
    }
    if (IV && a.iv_out) {  // final chain block of each payload ending in this step
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
        dec_cbc<R>(lds, lo, dk0, c, d, si_bytes(a.tables));  // all R rows per LDS round trip (A/B: ~1% over 2 rows)
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
            dec_cbc<R>(lds, lo, dk0, c, d, si_bytes(a.tables));
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
                        dec_cbc<1>(lds, lo, dk, cc, dd, si_bytes(a.tables));
                        d[k] = dd[0];
                    }
                }
            }
        }
    }
    if (FULL && STRIDED) {
        // A scheduling boundary between the rounds and the row addresses: in one
        // region with them, the per-row address arithmetic tipped the scheduler
        // into a low-pressure schedule that issues the rounds' LDS reads 4-7 at
        // a time (318 s_waitcnt per 640 reads against 53 in 64-read bursts), and
        // the strided step ran 4-5 % slower than the contiguous one on the same
        // bytes (profiles/r05/ab_dec_sched_barrier.txt).
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < R; k++) ST16U(probe_dec_addr<2>(out_s, srow<BIG>(a, ps, lane, k, rk, pk), lane), oe, d[k]);
    } else if (FULL) {
        uint8_t* o0 = a.out + 16 * (base + lane);
#pragma unroll
        for (int k = 0; k < R; k++) ST16(o0 + 1024 * k, oe, d[k]);
    } else {
#pragma unroll
        for (int k = 0; k < R; k++) {
            const uint64_t g = base + 64 * k + lane;
            if (g < end) {
                if (STRIDED) ST16U(a.out + soff_g(a, g), oe, d[k]);
                else ST16(a.out + 16 * g, oe, d[k]);
            }
        }
    }
    return make_uint4(rl63(c[R - 1].x), rl63(c[R - 1].y), rl63(c[R - 1].z), rl63(c[R - 1].w));  // next carry
}

// In-place launches with static ranges hand each range's carry C[begin-1]
// over without a prepass (DecArgs.handoff = the launch's epoch, unique in the
// process; boundary = one 32-B record per range: the block, then the epoch).
// Before its first store, a wave publishes for each of its ranges t the last
// ciphertext block C[end-1] -- still ciphertext: only this wave writes it --
// into record t+1, then the epoch, each store completed before the next
// access, so the epoch is visible before any plaintext of the range.  Then,
// for each of its ranges that starts inside a payload, it loads C[begin-1]
// from the stream and, once that load has completed, the record's epoch:
// published, the record holds the block; not published, range t-1's wave has
// not stored anything yet, so the loaded block is ciphertext and the wave
// writes it into the record itself (a writer arriving later writes the same
// bytes).  Neither side waits for the
// other, so nothing assumes the waves are resident together.  The range loop
// then reads its carry from the record, as from the prepass's snapshot.
template <bool STRIDED>
__device__ __forceinline__ uint4 dec_blk_at(const DecArgs& a, const uint8_t* in, uint64_t nblocks, uint64_t g) {
    if (STRIDED) return LD16U(a.in + soff_g(a, g), data_ext(a.in, a, true));
    return LD16(in + 16 * g, ext(in, 16 * nblocks));
}
// The records are written and read with agent-scope relaxed atomics (coherent
// across the XCDs' L2s without writing back or invalidating them), ordered by
// waits for the wave's own memory accesses to complete (vm_drain; the
// workgroup-scope fence emits none between two stores): an agent-scope fence
// here writes back and invalidates the whole L2 at every wave's start
// (measured +5 % on a relay-sized in-place decrypt).
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // s_waitcnt vmcnt(0) (gfx9 encoding)
__device__ __forceinline__ void rec_store(uint4* r, uint4 v) {
    uint32_t* w = reinterpret_cast<uint32_t*>(r);
    __hip_atomic_store(w + 0, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(w + 1, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(w + 2, v.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(w + 3, v.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint4 rec_load(const uint4* r) {
    uint32_t* w = const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(r));
    return make_uint4(__hip_atomic_load(w + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                      __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                      __hip_atomic_load(w + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                      __hip_atomic_load(w + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
template <bool STRIDED>
__device__ __forceinline__ void dec_handoff(const DecArgs& a, uint64_t wave, uint64_t nwaves, uint32_t lane) {
    uint4* rec = const_cast<uint4*>(a.boundary);
    const uint64_t nblocks = a.nblocks, epoch = a.handoff, len = a.stat_blocks;
    const uint32_t bpp = a.bpp.d;
    const Ext re = ext(rec, 32ull * a.nranges);
    for (uint64_t t = wave; t < a.nstat; t += nwaves) {
        const uint64_t end = min((t + 1) * len, nblocks);
        if (end >= nblocks || end % bpp == 0) continue;  // range t + 1 starts a payload (or does not exist)
        const uint4 last = dec_blk_at<STRIDED>(a, a.in, nblocks, end - 1);
        if (lane == 0) rec_store(AT(rec + 2 * (t + 1), re, 16), last);
        vm_drain();  // the block before the epoch
        if (lane == 0)
            __hip_atomic_store(reinterpret_cast<uint64_t*>(AT(rec + 2 * (t + 1) + 1, re, 8)), epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        vm_drain();  // the epoch before any plaintext store
    }
    for (uint64_t t = wave; t < a.nstat; t += nwaves) {
        const uint64_t begin = t * len;
        if (begin == 0 || begin % bpp == 0) continue;  // starts a payload: no carry
        const uint4 prev = dec_blk_at<STRIDED>(a, a.in, nblocks, begin - 1);
        vm_drain();  // the block loaded before the epoch is
        const uint64_t e = __hip_atomic_load(reinterpret_cast<uint64_t*>(AT(rec + 2 * t + 1, re, 8)), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        if (e != epoch && lane == 0) rec_store(AT(rec + 2 * t, re, 16), prev);
    }
    vm_drain();  // the records as the range loop will read them
}

// SESS: sessions of payloads_per_key payloads that are whole steps long
// (a.sess_blocks, a multiple of 64 * R; config D: 256 x 92 blocks) and whole
// ranges long: no range straddles two sessions, so the unkeyed step runs under
// a schedule chosen per range from the scalar block position, and no lane
// computes a key index.
// IV = false: no IV arrays (the relay's calls, cyr_rijndael.cpp:612 with iv =
// nullptr); the IV code and the payload-index tracking compile out, which
// keeps the SGPR budget of the round loop (with them, the !BIG SESS kernel
// scheduled its rounds with 321 s_waitcnt per 640 LDS reads against 173).
// DIV: the progress-feedback divisor (steps behind the workgroup's leader per
// priority level): kDecPrioDiv for long launches, kDecPrioDivShort when each
// wave has few steps (the runtime's choice, DecArgs / launch_decrypt_flat).
// The walk itself, after the decrypt image is in LDS and the workgroup's
// progress word (*leadp, in the launch's work words) is zero.  KOFF: the byte
// offset of these DecArgs inside the kernel's argument segment (0 for
// k_decrypt_flat; the duplex kernel's arguments start with its EncArgs).
// XW: the XCD-weighted static split (A/B, DecArgs.xw) -- its own instantiation:
// compiled into the others, the range code broke their LDS schedule (s_waitcnt
// 232 -> 493 per step body, relay-stream decrypt +7.8 %).
template <bool KEYED, bool BIG, bool SESS, bool IV, bool STRIDED, uint32_t DIV, uint32_t KOFF, bool XW = false>
__device__ __forceinline__ void dec_flat_body(const DecArgs& a, const char* lds, uint32_t* leadp) {
    constexpr int R = kDecRows;
    uint32_t prog = 0;
    const uint64_t wave =
        (uint64_t)blockIdx.x * (kDecThreads / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lo = dec_lo(threadIdx.x);
    uint32_t dk0[44];
    uint32_t dk_id = 0;  // KEYED: session whose schedule dk0 holds (~0u: none yet)
    if (KEYED) dk_id = ~0u;
    else if (!SESS) load_sched(a.keys, 0, 1, dk0);
    // Work ranges (DecArgs): wave w first takes static range w, then (dyn)
    // ranges of the dynamic pool from the per-XCD ticket pools, stealing from
    // the other XCDs' pools when its own is exhausted, so waves on faster CUs
    // and XCDs take more; or (static only) ranges w + nwaves, ...  KEYED
    // (per-lane keys) and IV (IV arrays): one static range per wave, as the
    // runtime launches them (the range loop around their larger step bodies
    // cost VGPR spills).
    const uint32_t nwaves = gridDim.x * (kDecThreads / 64);
    if (a.handoff) dec_handoff<STRIDED>(a, wave, nwaves, lane);
    uint32_t pool = xcc_id();
    uint32_t ticket = (uint32_t)wave;
    if (a.dyn && ticket >= a.nstat)
        ticket = a.nstat + dyn_ticket(a.work, pool, a.per_xcd, (uint32_t)a.nranges - a.nstat);
    while (true) {
        // The range's parameters are re-read from the kernel arguments here (an
        // opaque pointer keeps the loads in this block) instead of being held in
        // SGPRs across the step loop: with them live there the SGPR budget ran
        // out and the compiler scheduled the steps with 320 s_waitcnt per 640
        // LDS reads instead of 53.
        KernArg<DecArgs> ka = (KernArg<DecArgs>)((const __attribute__((address_space(4))) char*)
                                                     __builtin_amdgcn_kernarg_segment_ptr() + KOFF);
        asm volatile("" : "+s"(ka));
        if (ticket >= ka->nranges) break;
        const bool stat = ticket < ka->nstat;
        uint64_t begin = stat ? (uint64_t)ticket * ka->stat_blocks
                              : (uint64_t)ka->nstat * ka->stat_blocks + (uint64_t)(ticket - ka->nstat) * ka->range_blocks;
        uint64_t end = min(begin + (stat ? ka->stat_blocks : ka->range_blocks), ka->nblocks);
        if constexpr (XW) {  // (A/B) the XCD-weighted split: this wave's one range in its slot's span
            const uint32_t x = blockIdx.x % kXcds, wpx = nwaves / kXcds;
            const uint64_t idx = (uint64_t)(blockIdx.x / kXcds) * (kDecThreads / 64) + (wave % (kDecThreads / 64));
            uint64_t span0 = 0;
            for (uint32_t y = 0; y < x; y++) span0 += (uint64_t)wpx * ka->xsteps[y];
            const uint64_t len = (uint64_t)ka->xsteps[x] * (64 * R);
            begin = min(span0 * (64 * R) + idx * len, ka->nblocks);
            end = min(begin + len, ka->nblocks);
            if (begin >= end) break;
        }
        FlatPos ps;
        ps.bp = begin / a.bpp.d;
        ps.bpos = (uint32_t)(begin - ps.bp * a.bpp.d);
        uint4 carry = make_uint4(0, 0, 0, 0);  // C[begin-1]
        if (ps.bpos != 0) {  // (begin >= 1 here)
            if (ka->boundary && ka->handoff) carry = rec_load(AT(ka->boundary + 2 * ticket, ext(ka->boundary, 32ull * ka->nranges), 16));
            else if (ka->boundary) carry = LD16(ka->boundary + 2 * ticket, ext(ka->boundary, 32ull * ka->nranges));
            else if (STRIDED) carry = LD16U(a.in + soff(a, ps.bp, ps.bpos - 1), data_ext(a.in, a, true));
            else carry = LD16(ka->in + 16 * (begin - 1), ext(ka->in, 16 * ka->nblocks));
        }
        // SESS: a range lies in one session (the runtime makes range_blocks
        // divide sess_blocks); its schedule is loaded per range (11 loads per
        // range: tracking the current session kept one more SGPR live and the
        // compiler spilled VGPRs in the step loop).
        if (SESS) load_sched(a.keys, (uint32_t)(begin / ka->sess_blocks), 1, dk0);
        // !BIG: each lane tracks its rows' positions in their payloads, advanced
        // by step_r per step (one add and a min instead of a division per row).
        // STRIDED: row 0's position and payload only (srow_pos derives the rest)
        uint32_t rk[R], pk[R];
        if (!BIG) {
#pragma unroll
            for (int k = 0; k < (STRIDED ? 1 : R); k++) {
                const uint32_t lpos = ps.bpos + 64 * k + lane;
                const Fastdiv bd = {ka->bpp.M, ka->bpp.d};
                const uint32_t q = fastdiv(lpos, bd);
                rk[k] = lpos - q * bd.d;
                if (STRIDED) pk[k] = (uint32_t)(ps.bp + q) * (uint32_t)ka->stride + 16u * rk[k];  // row 0's offset
            }
        }
        auto advance = [&] {
            ps.bpos += a.step_r;
            ps.bp += a.step_q;
            if (ps.bpos >= a.bpp.d) { ps.bpos -= a.bpp.d; ps.bp++; }
            if (STRIDED) {  // wave-uniform: keep it in SGPRs (the compiler moved it to a VGPR pair)
                ps.bp = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(ps.bp >> 32)) << 32) |
                        __builtin_amdgcn_readfirstlane((uint32_t)ps.bp);
                ps.bpos = __builtin_amdgcn_readfirstlane(ps.bpos);
            }
            if (!BIG) {
#pragma unroll
                for (int k = 0; k < (STRIDED ? 1 : R); k++) {
                    const uint32_t t = rk[k] + a.step_r;  // < 2 bpp
                    if (STRIDED)  // 64 R blocks on, and the gap of each payload start passed
                        pk[k] += 1024u * R + (a.step_q + (t >= a.bpp.d ? 1u : 0u)) * ((uint32_t)a.stride - 16u * a.bpp.d);
                    rk[k] = min(t, t - a.bpp.d);
                }
            }
        };
        // STRIDED: the range's base pointers with off0 folded in (kernel arguments, re-read per range)
        const uint8_t* in_s = STRIDED ? ka->in + ka->off0 : nullptr;
        uint8_t* out_s = STRIDED ? ka->out + ka->off0 : nullptr;
        uint64_t base = begin;
        uint4 c[R], pv[R];
        if (base + 64 * R <= end) flat_load<true, BIG, STRIDED>(a, in_s, lane, base, end, ps, rk, pk, c, pv);
        for (; base + 64 * R <= end; base += 64 * R) {
            // (Issuing the next step's loads before this step's rounds measured ~1 %
            // slower: the LDS binds, and the other 15 waves hide the loads.)
            carry = flat_step<KEYED, BIG, true, IV, STRIDED>(a, lds, lo, lane, base, end, ps, carry, dk0, dk_id, c, pv,
                                                             rk, pk, out_s);
            if (STRIDED) {  // the next step's addresses come from its positions
                advance();
                if (base + 128 * R <= end)
                    flat_load<true, BIG, STRIDED>(a, in_s, lane, base + 64 * R, end, ps, rk, pk, c, pv);
                prio_feedback(leadp, ++prog, DIV);
            } else {
                if (base + 128 * R <= end)
                    flat_load<true, BIG, STRIDED>(a, in_s, lane, base + 64 * R, end, ps, rk, pk, c, pv);
                prio_feedback(leadp, ++prog, DIV);
                advance();
            }
        }
        if (base < end) {  // the batch's last, partial step (only the last range has one)
            flat_load<false, BIG, STRIDED>(a, in_s, lane, base, end, ps, rk, pk, c, pv);
            flat_step<KEYED, BIG, false, IV, STRIDED>(a, lds, lo, lane, base, end, ps, carry, dk0, dk_id, c, pv, rk, pk,
                                                      out_s);
        }
        if (KEYED || IV) break;
        ticket = ka->dyn ? ka->nstat + dyn_ticket(ka->work, pool, ka->per_xcd, (uint32_t)ka->nranges - ka->nstat)
                         : ticket + nwaves;
    }
}

}  // namespace
}  // namespace cyaes
