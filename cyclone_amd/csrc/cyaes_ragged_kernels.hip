// cyaes_ragged_kernels.hip -- gfx950 CBC decrypt of ragged batches
// (k_decrypt_ragged; cyr_rijndael.cpp:612-635 + _decryptBlock :708-774): the
// payloads of a device offset / size list, in groups packed into wave rows;
// and the flat decrypt's per-payload-key instantiations (k_decrypt_flat_keyed).
// Its own translation unit since r05, compiled with the iterative ILP scheduler
// (Makefile SCHED_RAG): under the default scheduler of cyaes_kernels.hip the
// step issued its LDS reads 4-8 at a time; moved here with a scheduling
// boundary before the stores, the relay-stream decrypt through the ragged
// entry points takes -2.8 % (profiles/r05/ab_ragged_sched.txt), while the quad
// encrypt left in cyaes_kernels.hip measured +4 % under this scheduler.
#define CYAES_TU 4
#include "cyaes_dec_body.h"

namespace cyaes {
namespace {

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

#ifndef CYAES_RAG_FULL_STEPS
#define CYAES_RAG_FULL_STEPS 1  // 0: A/B variant, a regular group's full steps through the selects and masks too
#endif
#ifndef CYAES_DEC_RAGGED_DIV
// The progress-feedback divisor: the short-launch one (a relay stream's ragged
// decrypt has ~92 steps per wave; r06 A/B at 8 / 4 / 2: 1.161 / 1.153 / 1.144
// ms, profiles/r06/ab3/ragdiv.txt).
#define CYAES_DEC_RAGGED_DIV kDecPrioDivShort
#endif
template <bool KEYED>
__global__ __launch_bounds__(kDecThreads, 1) void k_decrypt_ragged(DecArgs a) {
    constexpr int R = kDecRows;
    __shared__ __attribute__((aligned(16))) uint32_t lds_words[kDecLdsWords];
    fill_dec_image(lds_words, a.tables);
    uint32_t* leadp = dec_lead_word(a.work);
    if (threadIdx.x == 0) *leadp = 0;
    uint32_t prog = 0;
    __syncthreads();
    CLOCK_PROBE(1);
    const char* lds = reinterpret_cast<const char*>(lds_words);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lo = dec_lo(threadIdx.x);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t wave0 =
        (uint64_t)blockIdx.x * (blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t G = a.group;
    const uint64_t ngroups = a.nranges;  // (npayloads + G - 1) / G
    const Ext iv_in_e = iv_ext(a.iv_in, a.npayloads), iv_out_e = iv_ext(a.iv_out, a.npayloads);
    uint32_t dk0[44];
    uint32_t dk_id = ~0u;  // session whose schedule dk0 holds
    if (!KEYED) {
        load_sched(a.keys, 0, 1, dk0);
        dk_id = 0;
    }
    // Groups [0, nstat) are static (wave w takes w, w + nwaves, ...); then (dyn)
    // groups nstat + t of the dynamic pool from the per-XCD ticket pools, with
    // stealing (cyaes_device.h, dyn_ticket), so the waves and XCDs finish together.
    uint32_t pool = xcc_id();
    const uint32_t nst = a.dyn ? a.nstat : (uint32_t)ngroups;
    const uint32_t ndyn = (uint32_t)ngroups - nst;
    uint64_t grp = wave0;
    if (grp >= nst) grp = a.dyn ? nst + dyn_ticket(a.work, pool, a.per_xcd, ndyn) : ngroups;
    for (; grp < ngroups;) {
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
        // (r06) A regular group's rows are addressed as 32-bit offsets from its
        // first payload (a scalar base), advanced by an add per row plus the
        // packet gap at a payload boundary, as the flat kernel's strided rows
        // are: no 64-bit multiply-add per row.  Groups spanning 4 GiB or more
        // take the general path.
        const bool regular = nb0 >= 64 && (uint64_t)gn * ostr < (1ull << 32) &&
                             __ballot(holder && (nbh != nb0 || offh != off0 + (uint64_t)lane * ostr)) == 0;
        uint32_t jt = 0, rt = lane - 64u;  // regular: this lane's payload and block; the first row adds 64
        uint32_t ro = 16u * (lane - 64u);  // regular: jt * ostr + 16 rt, mod 2^32
        const uint32_t gap = (uint32_t)ostr - 16u * nb0;  // regular: bytes from a payload's end to the next one's start
        const uint8_t* gin = a.in + off0;  // regular: the group's first payload (wave-uniform)
        uint8_t* gout = a.out + off0;
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
            uint32_t o32[R];
            bool valid[R];
#pragma unroll
            for (int k = 0; k < R; k++) {
                if (regular) {
                    rt += 64;
                    ro += 1024u;
                    if (rt >= nb0) rt -= nb0, jt++, ro += gap;
                    valid[k] = jt < gn;
                    rr[k] = rt;
                    jr[k] = jt;
                    o32[k] = ro;
                    orow[k] = 0;
                    continue;
                }
                o32[k] = 0;
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
            // A full step of a regular group (every step but a group's last): every lane valid,
            // loads and stores without selects or exec masks.
            const bool rfull = CYAES_RAG_FULL_STEPS && regular && base + 64 * R <= total;
            if (rfull) {
#pragma unroll
                for (int k = 0; k < R; k++) c[k] = LD16U(gin + o32[k], re[k]);
            } else if (regular) {  // (as below: an invalid lane loads row 0 lane 0's block)
                const uint32_t safe32 = __builtin_amdgcn_readlane(o32[0], 0);
#pragma unroll
                for (int k = 0; k < R; k++) c[k] = LD16U(gin + (valid[k] ? o32[k] : safe32), re[k]);
            } else {
                const uint64_t safe = rlane64(orow[0], 0);
#pragma unroll
                for (int k = 0; k < R; k++) c[k] = LD16U(a.in + (valid[k] ? orow[k] : safe), re[k]);
            }
            // The progress atomic (a global word: the decrypt image fills the LDS) goes
            // out after the step's loads, so its round trip overlaps theirs instead of
            // delaying them (A/B: -1 % on relay streams, profiles/r02/ab_ragged_prio_late.txt).
            prio_feedback(leadp, ++prog, CYAES_DEC_RAGGED_DIV);
            pv[0] = shr1(c[0], carry);
#pragma unroll
            for (int k = 1; k < R; k++)
                pv[k] = shr1(c[k], make_uint4(rl63(c[k - 1].x), rl63(c[k - 1].y), rl63(c[k - 1].z), rl63(c[k - 1].w)));
            if (!a.iv_in && !a.iv_out) {  // relay streams: restarts at DefaultIV, a select per row
#pragma unroll
                for (int k = 0; k < R; k++)
                    if (rr[k] == 0) pv[k] = default_iv();
            } else {
#pragma unroll
                for (int k = 0; k < R; k++) {
                    const uint64_t p = p0 + jr[k];
                    if (valid[k] && rr[k] == 0) pv[k] = a.iv_in ? LD16(a.iv_in + 16 * p, iv_in_e) : default_iv();
                    if (a.iv_out) {  // (uniform branch: every lane runs the bpermute; one from an inactive lane reads 0)
                        const uint32_t nbj = regular ? nb0 : bperm(nbh, jr[k]);
                        if (valid[k] && rr[k] + 1 == nbj) ST16(a.iv_out + 16 * p, iv_out_e, c[k]);
                    }
                }
            }
            if (!KEYED) {
                dec_cbc<R>(lds, lo, dk0, c, pv, si_bytes(a.tables));
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
                    dec_cbc<R>(lds, lo, dk0, c, pv, si_bytes(a.tables));
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
                                dec_cbc<1>(lds, lo, dk, cc, dd, si_bytes(a.tables));
                                pv[k] = dd[0];
                            }
                        }
                    }
                }
            }
            // A scheduling boundary between the rounds and the stores: in one
            // region with the stores' 64-bit row offsets the rounds' LDS reads
            // went out 4-8 at a time (320 / 158 s_waitcnt per 640 reads); with
            // it, and this TU's iterative-ILP scheduler, in bursts of 64 (13 / 31).
            __builtin_amdgcn_sched_barrier(0);
            if (rfull) {
#pragma unroll
                for (int k = 0; k < R; k++) {
                    Ext we = re[k];
                    if constexpr (CYAES_BOUNDS_CHECK) we = ext(a.out + (we.lo - a.in), we.hi - we.lo);
                    ST16U(gout + o32[k], we, pv[k]);
                }
            } else {
#pragma unroll
                for (int k = 0; k < R; k++) {
                    Ext we = re[k];
                    if constexpr (CYAES_BOUNDS_CHECK) we = ext(a.out + (we.lo - a.in), we.hi - we.lo);
                    if (valid[k]) ST16U(regular ? gout + o32[k] : a.out + orow[k], we, pv[k]);
                }
            }
            carry = make_uint4(rl63(c[R - 1].x), rl63(c[R - 1].y), rl63(c[R - 1].z), rl63(c[R - 1].w));
        }
        // next group: static ones by stride, then the dynamic pool
        const uint64_t nxt = grp + nwaves;
        grp = nxt < nst ? nxt : (a.dyn ? nst + dyn_ticket(a.work, pool, a.per_xcd, ndyn) : ngroups);
    }
}

// The flat decrypt with per-payload keys (key index arrays, sessions that are
// not whole steps; with IV arrays): under the decrypt unit's max-ILP scheduler
// its step issued the LDS reads 4-7 at a time (320 s_waitcnt per 640 reads),
// here in bursts of 64 (13): config D's sessions given as a key index array
// decrypt -8.5 % (profiles/r05/ab_dec_keyed_sched.txt).  The other flat
// instantiations stay in cyaes_dec_kernels.hip, where the strided one keeps
// its registers (6 VGPR spills under this scheduler, +1 %).
template <bool BIG>
__global__ __launch_bounds__(kDecThreads, 1) void k_decrypt_flat_keyed(DecArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_words[kDecLdsWords];
    fill_dec_image(lds_words, a.tables);
    uint32_t* leadp = dec_lead_word(a.work);
    if (threadIdx.x == 0) *leadp = 0;
    __syncthreads();
    CLOCK_PROBE(1);
    dec_flat_body<true, BIG, false, true, false, kDecPrioDiv, 0>(a, reinterpret_cast<const char*>(lds_words), leadp);
}

}  // namespace

void launch_decrypt_flat_keyed(const DecArgs& a, dim3 g, dim3 b, hipStream_t stream) {
    if (a.bpp.d >= 64u * kDecRows) hipLaunchKernelGGL(k_decrypt_flat_keyed<true>, g, b, 0, stream, a);
    else hipLaunchKernelGGL(k_decrypt_flat_keyed<false>, g, b, 0, stream, a);
}

hipError_t launch_decrypt_ragged(const DecArgs& a, int grid, int threads, hipStream_t stream) {
    const bool keyed = a.keys.key_idx != nullptr || a.keys.ppk.d != 0;
    if (keyed) hipLaunchKernelGGL(k_decrypt_ragged<true>, dim3(grid), dim3(threads), 0, stream, a);
    else hipLaunchKernelGGL(k_decrypt_ragged<false>, dim3(grid), dim3(threads), 0, stream, a);
    return hipGetLastError();
}

#if CYAES_BOUNDS_CHECK
int bounds_read_rag(unsigned long long* rec4, unsigned int* lines) { return read_bounds_local(rec4, lines); }
#endif
#if CYAES_CLOCK_PROBE
int probe_read_rag(unsigned long long* out8) { return read_probe_local(out8); }
int timeline_read_rag(int kind, uint4* out) { return read_timeline_local(kind, out); }
#endif

}  // namespace cyaes
