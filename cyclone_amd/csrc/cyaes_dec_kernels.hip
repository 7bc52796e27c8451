// cyaes_dec_kernels.hip -- gfx950 CBC decrypt of uniform contiguous batches,
// one lane per block (k_decrypt_flat; cyr_rijndael.cpp:612-635 + _decryptBlock
// :708-774).  Compiled with the max-ILP scheduler (Makefile SCHED_DEC): config
// C decrypt -1.5 % (profiles/r03/ab_sched.txt); design notes in cyaes_kernels.hip
// and DESIGN.md §3.3.

#define CYAES_TU 2
#include "cyaes_dec_body.h"

namespace cyaes {
namespace {

template <bool KEYED, bool BIG, bool SESS, bool IV, bool STRIDED, uint32_t DIV, bool XW = false>
__global__ __launch_bounds__(kDecThreads, 1) void k_decrypt_flat(DecArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_words[kDecLdsWords];
    fill_dec_image(lds_words, a.tables);
    uint32_t* leadp = dec_lead_word(a.work);
    if (threadIdx.x == 0) *leadp = 0;
    __syncthreads();
    CLOCK_PROBE(1);
    dec_flat_body<KEYED, BIG, SESS, IV, STRIDED, DIV, 0, XW>(a, reinterpret_cast<const char*>(lds_words), leadp);
}

// Before a decrypt (one small launch, stream-ordered): zero the launch's work
// words, and for an in-place flat decrypt snapshot C[begin-1] of every range
// before any wave overwrites it.
__global__ void k_dec_prepass(DecArgs a, uint32_t work_words) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < work_words) a.work[r] = 0;
    if (!a.boundary || r >= a.nranges) return;
    const uint64_t begin = r < a.nstat ? r * a.stat_blocks : a.nstat * a.stat_blocks + (r - a.nstat) * a.range_blocks;
    if (begin == 0 || begin >= a.nblocks || begin % a.bpp.d == 0) return;
    uint4* snap = const_cast<uint4*>(a.boundary) + 2 * r;  // (32-B records: dec_handoff's layout)
    const Ext se = ext(a.boundary, 32 * a.nranges);
    if (a.stride) ST16(snap, se, LD16U(a.in + soff_g(a, begin - 1), data_ext(a.in, a, true)));
    else ST16(snap, se, LD16(a.in + 16 * (begin - 1), ext(a.in, 16 * a.nblocks)));
}

}  // namespace

template <uint32_t DIV>
static void launch_flat(const DecArgs& a, dim3 g, dim3 b, hipStream_t stream) {
    const bool keyed = a.keys.key_idx != nullptr || a.keys.ppk.d != 0;
    const bool big = a.bpp.d >= 64u * kDecRows;
    const bool sess = a.sess_blocks != 0;  // keyed by step-aligned sessions: the unkeyed step per session
    const bool iv = a.iv_in != nullptr || a.iv_out != nullptr;  // (the runtime sets sess only without IVs)
    // STRIDED: unkeyed, no IV arrays (the runtime checks)
    if (a.xw && big) hipLaunchKernelGGL((k_decrypt_flat<false, true, false, false, false, DIV, true>), g, b, 0, stream, a);
    else if (a.xw) hipLaunchKernelGGL((k_decrypt_flat<false, false, false, false, false, DIV, true>), g, b, 0, stream, a);
    else if (a.stride && big) hipLaunchKernelGGL((k_decrypt_flat<false, true, false, false, true, DIV>), g, b, 0, stream, a);
    else if (a.stride) hipLaunchKernelGGL((k_decrypt_flat<false, false, false, false, true, DIV>), g, b, 0, stream, a);
    else if (sess && big) hipLaunchKernelGGL((k_decrypt_flat<false, true, true, false, false, DIV>), g, b, 0, stream, a);
    else if (sess) hipLaunchKernelGGL((k_decrypt_flat<false, false, true, false, false, DIV>), g, b, 0, stream, a);
    else if (keyed) launch_decrypt_flat_keyed(a, g, b, stream);  // (cyaes_ragged_kernels.hip: iterative ILP)
    else if (big && iv) hipLaunchKernelGGL((k_decrypt_flat<false, true, false, true, false, kDecPrioDiv>), g, b, 0, stream, a);
    else if (big) hipLaunchKernelGGL((k_decrypt_flat<false, true, false, false, false, DIV>), g, b, 0, stream, a);
    else if (iv) hipLaunchKernelGGL((k_decrypt_flat<false, false, false, true, false, kDecPrioDiv>), g, b, 0, stream, a);
    else hipLaunchKernelGGL((k_decrypt_flat<false, false, false, false, false, DIV>), g, b, 0, stream, a);
}

hipError_t launch_decrypt_flat(const DecArgs& a, int grid, hipStream_t stream) {
    const dim3 g(grid), b(kDecThreads);
    if (a.prio_short) launch_flat<kDecPrioDivShort>(a, g, b, stream);
    else launch_flat<kDecPrioDiv>(a, g, b, stream);
    return hipGetLastError();
}

hipError_t launch_dec_prepass(const DecArgs& a, uint32_t work_words, hipStream_t stream) {
    const int threads = 256;
    const uint64_t n = std::max<uint64_t>(work_words, a.boundary ? a.nranges : 0);
    const int grid = (int)((n + threads - 1) / threads);
    hipLaunchKernelGGL(k_dec_prepass, dim3(grid), dim3(threads), 0, stream, a, work_words);
    return hipGetLastError();
}

#if CYAES_BOUNDS_CHECK
int bounds_read_dec(unsigned long long* rec4, unsigned int* lines) { return read_bounds_local(rec4, lines); }
#endif
#if CYAES_CLOCK_PROBE
int probe_read_dec(unsigned long long* out8) { return read_probe_local(out8); }
int timeline_read_dec(int kind, uint4* out) { return read_timeline_local(kind, out); }
#endif

}  // namespace cyaes
