// cyaes_adler.hip -- Adler-32 on gfx950 (include/cyaes_adler32.h).
//
// Reference: thejinchao/cyclone source/cyCrypt/crypt/cyr_adler32.cpp:66-133
// (zlib's update).  For a buffer x[0..n) and running value (a0, b0):
//     A = a0 + S,          S = sum x_i
//     B = b0 + n*a0 + n*S - T,   T = sum i*x_i      (all mod 65521)
// which is what the reference's sequential loop computes (its periodic MODs
// keep the same residues).  Both sums are position-independent partials, so
// any number of lanes can take any slices: per 16-B vector, four
// v_dot4_u32_u8 give the byte sums and four more the in-dword weights.
// Edge rules kept from the reference: len == 0 (or NULL) -> 1 (:72-73);
// len == 1 uses its two conditional subtractions (:80-87), which differ from
// a true modulo only for running values outside [0, 65521).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cyaes_adler32.h"

namespace cyaes {
namespace {

constexpr uint32_t kBase = 65521;
constexpr uint32_t kOnes = 0x01010101u, kIdx = 0x03020100u;

__device__ __forceinline__ uint32_t dot(uint32_t x, uint32_t w, uint32_t acc) {
    return __builtin_amdgcn_udot4(x, w, acc, false);
}

struct Part {  // partial sums of a slice, S = sum x, T = sum (global index) * x, both kept < 2^63
    uint64_t s = 0, t = 0;
};

// 16-B vector whose first byte has buffer index i (im = i mod kBase).
__device__ __forceinline__ void add_vec(Part& p, uint4 v, uint32_t im) {
    const uint32_t s0 = dot(v.x, kOnes, 0), s1 = dot(v.y, kOnes, 0), s2 = dot(v.z, kOnes, 0), s3 = dot(v.w, kOnes, 0);
    const uint32_t s = s0 + s1 + s2 + s3;
    uint32_t k = dot(v.x, kIdx, 0);
    k = dot(v.y, kIdx, k + 4 * s1);
    k = dot(v.z, kIdx, k + 8 * s2);
    k = dot(v.w, kIdx, k + 12 * s3);
    p.s += s;
    p.t += (uint64_t)im * s + k;
}

__device__ __forceinline__ void add_byte(Part& p, uint32_t x, uint64_t i) {
    p.s += x;
    p.t += (i % kBase) * x;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Adler-32 of n bytes with running value `adler`, from the slice sums.
__device__ __forceinline__ uint32_t finish(uint32_t adler, uint64_t n, uint64_t s, uint64_t t, uint32_t first_byte) {
    if (n == 0) return CYAES_INITIAL_ADLER;
    uint32_t a = adler & 0xffff, b = adler >> 16;
    if (n == 1) {  // cyr_adler32.cpp:80-87, verbatim arithmetic
        a += first_byte;
        if (a >= kBase) a -= kBase;
        b += a;
        if (b >= kBase) b -= kBase;
        return a | (b << 16);
    }
    const uint64_t nm = n % kBase, sm = s % kBase, tm = t % kBase, am = a % kBase;
    const uint32_t A = (uint32_t)((am + sm) % kBase);
    const uint64_t B = ((uint64_t)(b % kBase) + nm * am + nm * sm + (kBase - tm)) % kBase;
    return A | ((uint32_t)B << 16);
}

// Slice [lo, hi) of the buffer, in bytes; vectors from the first 16-B
// aligned address; lane `l` of `nl` takes every nl-th vector.
__device__ __forceinline__ Part slice(const uint8_t* buf, uint64_t n, uint64_t l, uint64_t nl) {
    Part p;
    const uint64_t head = (16 - ((uintptr_t)buf & 15)) & 15;
    const uint64_t h = head < n ? head : n;
    const uint64_t nvec = (n - h) / 16;
    const uint64_t tail0 = h + 16 * nvec;
    if (l < h) add_byte(p, buf[l], l);
    if (l < n - tail0) add_byte(p, buf[tail0 + l], tail0 + l);
    const uint4* v = reinterpret_cast<const uint4*>(buf + h);
    // im = (h + 16 * j) mod kBase, advanced by 16 * nl per step
    const uint32_t step = (uint32_t)((16 * nl) % kBase);
    uint32_t im = (uint32_t)((h + 16 * l) % kBase);
    auto adv = [&]() {
        im += step;
        if (im >= kBase) im -= kBase;
    };
    uint64_t j = l;
    for (; j + 3 * nl < nvec; j += 4 * nl) {  // four independent loads in flight per lane
        const uint4 a = v[j], b = v[j + nl], c = v[j + 2 * nl], d = v[j + 3 * nl];
        add_vec(p, a, im);
        adv();
        add_vec(p, b, im);
        adv();
        add_vec(p, c, im);
        adv();
        add_vec(p, d, im);
        adv();
    }
    for (; j < nvec; j += nl) {
        add_vec(p, v[j], im);
        adv();
    }
    p.s %= kBase;
    p.t %= kBase;
    return p;
}

// One wave per buffer.
__global__ __launch_bounds__(256) void k_adler32_batch(const uint8_t* buf, const uint64_t* offsets,
                                                      const uint64_t* nbytes, const uint32_t* adler_in,
                                                      uint32_t* out, uint64_t n) {
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); k < n; k += waves) {
        const uint8_t* b = buf + offsets[k];
        const uint64_t len = nbytes[k];
        const Part p = slice(b, len, lane, 64);
        const uint64_t s = wave_sum(p.s), t = wave_sum(p.t);
        if (lane == 0) out[k] = finish(adler_in ? adler_in[k] : CYAES_INITIAL_ADLER, len, s, t, len ? b[0] : 0);
    }
}

// Whole-grid reduction of one buffer into acc[0..1] (S, T partial sums mod kBase each).
__global__ __launch_bounds__(256) void k_adler32_big(const uint8_t* buf, uint64_t n, unsigned long long* acc) {
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    const Part p = slice(buf, n, (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt);
    const uint64_t s = wave_sum(p.s), t = wave_sum(p.t);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&acc[0], (unsigned long long)s);
        atomicAdd(&acc[1], (unsigned long long)t);
    }
}

__global__ void k_adler32_finish(const uint8_t* buf, uint64_t n, uint32_t adler, const unsigned long long* acc,
                                 uint32_t* out) {
    out[0] = finish(adler, n, acc[0], acc[1], n ? buf[0] : 0);
}

int map_err(hipError_t e) { return e == hipSuccess ? 0 : (e == hipErrorOutOfMemory ? -3 : -2); }

}  // namespace
}  // namespace cyaes

extern "C" {

int cyaes_gpu_adler32_batch(const uint8_t* d_buf, const uint64_t* d_offsets, const uint64_t* d_nbytes,
                            const uint32_t* d_adler_in, uint32_t* d_out, uint64_t n, void* stream) {
    if (n == 0) return 0;
    if (!d_buf || !d_offsets || !d_nbytes || !d_out) return -1;  // CYAES_EINVAL
    const uint64_t want = (n + 3) / 4;  // 4 waves per 256-thread block
    const int grid = (int)(want < 8192 ? want : 8192);
    hipLaunchKernelGGL(cyaes::k_adler32_batch, dim3(grid), dim3(256), 0, (hipStream_t)stream, d_buf, d_offsets,
                       d_nbytes, d_adler_in, d_out, n);
    return cyaes::map_err(hipGetLastError());
}

int cyaes_gpu_adler32(const uint8_t* d_buf, uint64_t nbytes, uint32_t adler, uint32_t* out, void* stream) {
    if (!out || (nbytes && !d_buf)) return -1;
    if (nbytes == 0) {
        *out = CYAES_INITIAL_ADLER;  // cyr_adler32.cpp:72-73
        return 0;
    }
    hipStream_t s = (hipStream_t)stream;
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    // ~4 vectors per thread at least; at most 8 blocks of 256 per CU.
    const uint64_t vecs = nbytes / 16 + 1;
    uint64_t grid = (vecs + 1023) / 1024;
    if (grid > (uint64_t)cus * 8) grid = (uint64_t)cus * 8;
    unsigned long long* acc = nullptr;
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&acc), 16 + 16, s);
    if (e != hipSuccess) return cyaes::map_err(e);
    uint32_t* d_out = reinterpret_cast<uint32_t*>(acc + 2);
    e = hipMemsetAsync(acc, 0, 16, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(cyaes::k_adler32_big, dim3((unsigned)grid), dim3(256), 0, s, d_buf, nbytes, acc);
        hipLaunchKernelGGL(cyaes::k_adler32_finish, dim3(1), dim3(1), 0, s, d_buf, nbytes, adler, acc, d_out);
        e = hipGetLastError();
    }
    uint32_t h = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&h, d_out, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFreeAsync(acc, s);
    if (e == hipSuccess) *out = h;
    return cyaes::map_err(e);
}

}  // extern "C"
