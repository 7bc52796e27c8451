// cyaes_enc_kernels.hip -- gfx950 CBC encrypt, one lane per payload chain
// (k_encrypt; cyr_rijndael.cpp:588-609 + _encryptBlock :638-705).  Compiled
// with the iterative ILP scheduler (Makefile SCHED_ENC): config C encrypt
// -1.5 %, B -1.3 % (profiles/r03/ab_sched.txt); the design notes are in
// cyaes_kernels.hip and DESIGN.md §3.2.  Also the relay-stream encrypt that
// reads 64-B lines (k_encrypt_lines).

#define CYAES_TU 1
#include "cyaes_lines_body.h"

namespace cyaes {
namespace {

template <bool RAGGED, bool KEYED, bool RUNS, bool SESS>
__global__ __launch_bounds__(kEncThreads, 1) void k_encrypt(EncArgs a) {
    // The list k_encrypt_rag_lines handed back (a relay stream's is empty): no
    // table image for nothing (5.9 us a launch, profiles/r06/final).
    if (RAGGED && a.rest && *a.rest == 0) return;
    __shared__ __attribute__((aligned(16))) uint32_t lds_words[kEncLdsWords];
    fill_enc_image(lds_words, a.tables);
    __shared__ uint32_t lead;  // prio_feedback
    if (threadIdx.x == 0) lead = 0;
    __syncthreads();
    CLOCK_PROBE(0);
    enc_body<RAGGED, KEYED, RUNS, SESS>(a, reinterpret_cast<const char*>(lds_words), &lead);
}

// Strided batches of whole 1,024-payload groups read by 64-B lines
// (cyaes_lines_body.h).
__global__ __launch_bounds__(kEncThreads, 1) void k_encrypt_lines(EncArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_words[kEncLdsWords];
    fill_enc_image(lds_words, a.tables);
    __shared__ uint32_t lead;  // prio_feedback
    if (threadIdx.x == 0) lead = 0;
    __syncthreads();
    CLOCK_PROBE(0);
    lines_walk(a, reinterpret_cast<const char*>(lds_words), &lead);
}


// Ragged batches' whole 1,024-payload groups by lines (cyaes_lines_body.h,
// rag_lines_walk); the waves it hands back go to k_encrypt<RAGGED> next.
__global__ __launch_bounds__(kEncThreads, 1) void k_encrypt_rag_lines(EncArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_words[kEncLdsWords];
    fill_enc_image(lds_words, a.tables);
    __shared__ uint32_t lead;  // prio_feedback
    if (threadIdx.x == 0) lead = 0;
    __syncthreads();
    CLOCK_PROBE(0);
    __shared__ uint32_t mpos[kEncThreads];  // per wave: its payloads' positions (rag_lines_walk)
    rag_lines_walk(a, reinterpret_cast<const char*>(lds_words), &lead, mpos);
}

}  // namespace

hipError_t launch_encrypt_rag_lines(const EncArgs& a, int grid, int threads, hipStream_t stream) {
    hipLaunchKernelGGL(k_encrypt_rag_lines, dim3(grid), dim3(threads), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_encrypt_lines(const EncArgs& a, int grid, int threads, hipStream_t stream) {
    hipLaunchKernelGGL(k_encrypt_lines, dim3(grid), dim3(threads), 0, stream, a);
    return hipGetLastError();
}


hipError_t launch_encrypt(const EncArgs& a, int grid, int threads, hipStream_t stream) {
    const bool keyed = a.keys.key_idx != nullptr || a.keys.ppk.d != 0;
    const bool ragged = a.offsets != nullptr || a.stride != 0;
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

#if CYAES_BOUNDS_CHECK
int bounds_read_enc(unsigned long long* rec4, unsigned int* lines) { return read_bounds_local(rec4, lines); }
#endif
#if CYAES_CLOCK_PROBE
int probe_read_enc(unsigned long long* out8) { return read_probe_local(out8); }
int timeline_read_enc(int kind, uint4* out) { return read_timeline_local(kind, out); }
#endif

}  // namespace cyaes
