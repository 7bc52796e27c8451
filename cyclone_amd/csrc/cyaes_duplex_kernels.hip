// cyaes_duplex_kernels.hip -- gfx950 duplex launch: one uniform batch
// encrypted and another decrypted by ONE persistent grid (cyaes_gpu_duplex_uniform).
//
// The relay carries both directions of a pipe at once: relay_server.cpp:472
// encrypts target -> tunnel while :329 decrypts tunnel -> target (and
// relay_local.cpp:206 / :365 the same on the client).  Run as two launches,
// each launch ends on its own tail: the encrypt is one CBC chain per lane and
// a chain cannot be split, so the XCDs' clock spread (up to ~6 %) and the
// spread inside a workgroup leave CUs idle at its end (config B: last wave /
// mean wave 1.076, config C 1.028; profiles/r04/final2/timeline_B.txt,
// profiles/r04/timeline_global_counter_C_static.txt).  Here every workgroup
// first walks its share of the encrypt batch exactly as k_encrypt does
// (cyaes_enc_body.h, 128 KiB encrypt image), waits for its own 16 waves,
// refills its LDS with the 160 KiB decrypt image and then walks decrypt
// ranges exactly as k_decrypt_flat does (cyaes_dec_body.h) with the dynamic
// pool on: a workgroup that finished its encrypt early takes more of the
// decrypt's pool, so the encrypt's tail is filled with decrypt work and the
// launch ends within about one decrypt range on every CU.
//
// Both halves: unkeyed (one schedule each, any row of the context's table),
// no IV arrays (every payload its own chain from DefaultIV, as the relay
// calls it), uniform contiguous batches; the runtime checks and otherwise
// runs the two halves as separate launches.
#define CYAES_TU 3
#include <stddef.h>

#include "cyaes_dec_body.h"
#include "cyaes_enc_body.h"
#include "cyaes_lines_body.h"

namespace cyaes {
namespace {

// LINES: the relay-stream form (cyaes_gpu_duplex_strided): the encrypt half
// is a strided stream walked by 64-B lines (cyaes_lines_body.h, whole
// 1,024-payload groups) and the decrypt half a strided stream walked by the
// flat kernel's STRIDED rows.
template <bool ERUNS, bool DBIG, uint32_t DIV, bool LINES = false>
__global__ __launch_bounds__(kDecThreads, 1) void k_duplex(DuplexArgs x) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_words[kDecLdsWords];
    const char* lds = reinterpret_cast<const char*>(lds_words);
    if (x.e.npayloads) {
        // Phase 1: the encrypt batch.  Its image is 128 KiB; its progress word
        // sits in the LDS just past it.
        fill_enc_image(lds_words, x.e.tables);
        uint32_t* elead = lds_words + kEncLdsWords;
        if (threadIdx.x == 0) *elead = 0;
        __syncthreads();
        {
            CLOCK_PROBE(0);  // (probe builds: the encrypt phase as kind 0)
            if (LINES) lines_walk(x.e, lds, elead);
            else enc_body<false, false, ERUNS, false>(x.e, lds, elead);
        }
        __syncthreads();  // all 16 waves are done with the encrypt image
    }
    // Phase 2: the decrypt batch, ranges from the launch's pools.
    fill_dec_image(lds_words, x.d.tables);
    uint32_t* leadp = dec_lead_word(x.d.work);
    if (threadIdx.x == 0) *leadp = 0;
    __syncthreads();
    CLOCK_PROBE(1);  // (the decrypt phase as kind 1)
    dec_flat_body<false, DBIG, false, false, LINES, DIV, (uint32_t)offsetof(DuplexArgs, d)>(x.d, lds, leadp);
}

template <bool ERUNS, bool DBIG, bool LINES = false>
void launch_div(const DuplexArgs& x, dim3 g, dim3 b, hipStream_t stream) {
    if (x.d.prio_short) hipLaunchKernelGGL((k_duplex<ERUNS, DBIG, kDecPrioDivShort, LINES>), g, b, 0, stream, x);
    else hipLaunchKernelGGL((k_duplex<ERUNS, DBIG, kDecPrioDiv, LINES>), g, b, 0, stream, x);
}

}  // namespace

hipError_t launch_duplex_lines(const DuplexArgs& x, int grid, hipStream_t stream) {
    const dim3 g(grid), b(kDecThreads);
    if (x.d.bpp.d >= 64u * kDecRows) launch_div<false, true, true>(x, g, b, stream);
    else launch_div<false, false, true>(x, g, b, stream);
    return hipGetLastError();
}

hipError_t launch_duplex(const DuplexArgs& x, int grid, hipStream_t stream) {
    const dim3 g(grid), b(kDecThreads);
    const bool runs = x.e.run > 1;
    const bool big = x.d.bpp.d >= 64u * kDecRows;
    if (runs && big) launch_div<true, true>(x, g, b, stream);
    else if (runs) launch_div<true, false>(x, g, b, stream);
    else if (big) launch_div<false, true>(x, g, b, stream);
    else launch_div<false, false>(x, g, b, stream);
    return hipGetLastError();
}

#if CYAES_BOUNDS_CHECK
int bounds_read_dup(unsigned long long* rec4, unsigned int* lines) { return read_bounds_local(rec4, lines); }
#endif
#if CYAES_CLOCK_PROBE
int probe_read_dup(unsigned long long* out8) { return read_probe_local(out8); }
int timeline_read_dup(int kind, uint4* out) { return read_timeline_local(kind, out); }
#endif

}  // namespace cyaes
