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

#include <mutex>

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
// The 16-B aligned body is cut into chunks of kChunkVecs vectors; a wave
// streams whole chunks (grid-stride over chunks), 64 lanes x 4 vectors per
// step, as the batch kernel streams a 64 KiB fragment.  (Measured the same as
// a grid-stride over single vectors; what cost the first version 6 % was its
// per-call allocation, memset and atomics, see cyaes_gpu_adler32.)
constexpr uint64_t kChunkVecs = 4096;  // 64 KiB
__global__ __launch_bounds__(256) void k_adler32_big(const uint8_t* buf, uint64_t n, unsigned long long* part) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const uint64_t head = (16 - ((uintptr_t)buf & 15)) & 15;
    const uint64_t h = head < n ? head : n;
    const uint64_t nvec = (n - h) / 16;
    const uint64_t tail0 = h + 16 * nvec;
    Part p;
    if (wave == 0) {  // unaligned head and tail bytes
        if (lane < h) add_byte(p, buf[lane], lane);
        if (lane < n - tail0) add_byte(p, buf[tail0 + lane], tail0 + lane);
    }
    const uint4* v = reinterpret_cast<const uint4*>(buf + h);
    const uint64_t nchunks = (nvec + kChunkVecs - 1) / kChunkVecs;
    constexpr uint32_t kStep = (16 * 64) % kBase;  // im advance per lane step of 64 vectors
    for (uint64_t c = wave; c < nchunks; c += nwaves) {
        const uint64_t j0 = c * kChunkVecs, j1 = j0 + kChunkVecs < nvec ? j0 + kChunkVecs : nvec;
        uint32_t im = (uint32_t)((h + 16 * (j0 + lane)) % kBase);
        auto adv = [&]() {
            im += kStep;
            if (im >= kBase) im -= kBase;
        };
        uint64_t j = j0 + lane;
        for (; j + 3 * 64 < j1; j += 4 * 64) {  // four independent loads in flight per lane
            const uint4 a = v[j], b = v[j + 64], cc = v[j + 128], d = v[j + 192];
            add_vec(p, a, im);
            adv();
            add_vec(p, b, im);
            adv();
            add_vec(p, cc, im);
            adv();
            add_vec(p, d, im);
            adv();
        }
        for (; j < j1; j += 64) {
            add_vec(p, v[j], im);
            adv();
        }
        p.s %= kBase;
        p.t %= kBase;
    }
    const uint64_t s = wave_sum(p.s), t = wave_sum(p.t);
    if (lane == 0) {  // one (S, T) pair per wave, summed by k_adler32_finish (no memset, no atomics)
        part[2 * wave] = s % kBase;
        part[2 * wave + 1] = t % kBase;
    }
}

// Sums the per-wave partials (one block of 256 threads) and finishes.
__global__ __launch_bounds__(256) void k_adler32_finish(const uint8_t* buf, uint64_t n, uint32_t adler,
                                                       const unsigned long long* part, uint32_t nparts,
                                                       uint32_t* out) {
    uint64_t s = 0, t = 0;  // each partial < kBase: no overflow for any realistic count
    for (uint32_t w = threadIdx.x; w < nparts; w += blockDim.x) {
        s += part[2 * w];
        t += part[2 * w + 1];
    }
    s = wave_sum(s);
    t = wave_sum(t);
    __shared__ uint64_t ws[4], wt[4];
    if ((threadIdx.x & 63) == 0) {
        ws[threadIdx.x >> 6] = s;
        wt[threadIdx.x >> 6] = t;
    }
    __syncthreads();
    if (threadIdx.x == 0) out[0] = finish(adler, n, ws[0] + ws[1] + ws[2] + ws[3], wt[0] + wt[1] + wt[2] + wt[3],
                                          n ? buf[0] : 0);
}

constexpr int kMaxDevices = 64;
struct AdlerScratch {
    std::mutex mu;
    unsigned long long* part = nullptr;  // 2 words per wave of the largest grid, then the result word
    uint32_t* host = nullptr;            // pinned
    uint32_t max_grid = 0;
};
AdlerScratch g_adler_scratch[kMaxDevices];

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
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= cyaes::kMaxDevices) return -2;
    // Per-device scratch, made once: per-wave partials, the result word, a
    // pinned host word.  Calls on one device serialise on it (the call is synchronous anyway).
    cyaes::AdlerScratch& sc = cyaes::g_adler_scratch[dev];
    std::lock_guard<std::mutex> lock(sc.mu);
    if (!sc.part) {
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const uint32_t max_grid = (uint32_t)cus * 8;
        unsigned long long* part = nullptr;
        uint32_t* host = nullptr;
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&part), 16ull * 4 * max_grid + 16);
        if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&host), 4, hipHostMallocDefault);
        if (e != hipSuccess) {
            if (part) (void)hipFree(part);
            return cyaes::map_err(e);
        }
        sc.part = part;
        sc.host = host;
        sc.max_grid = max_grid;
    }
    // One wave per 64 KiB chunk up to 8 blocks of 4 waves per CU (grid-stride beyond).
    const uint64_t chunks = (nbytes / 16 + cyaes::kChunkVecs - 1) / cyaes::kChunkVecs + 1;
    uint64_t grid = (chunks + 3) / 4;
    if (grid > sc.max_grid) grid = sc.max_grid;
    const uint32_t nparts = (uint32_t)grid * 4;
    uint32_t* d_out = reinterpret_cast<uint32_t*>(sc.part + 2ull * 4 * sc.max_grid);
    hipLaunchKernelGGL(cyaes::k_adler32_big, dim3((unsigned)grid), dim3(256), 0, s, d_buf, nbytes, sc.part);
    hipLaunchKernelGGL(cyaes::k_adler32_finish, dim3(1), dim3(256), 0, s, d_buf, nbytes, adler, sc.part, nparts,
                       d_out);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(sc.host, d_out, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess) *out = *sc.host;
    return cyaes::map_err(e);
}

}  // extern "C"
