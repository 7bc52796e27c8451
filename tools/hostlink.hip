// tools/hostlink.hip -- how fast can gfx950 kernels move relay packets between
// pinned host memory and HBM themselves (the batcher's zero-copy gather /
// scatter), against the DMA engines (hipMemcpyAsync)?
//
// Measures, per pattern, GB/s (1e9 B/s) of payload moved:
//   dma_h2d / dma_d2h / dma_duplex : hipMemcpyAsync of one contiguous range
//   k_read / k_write / k_duplex   : a kernel streaming contiguous host memory
//   pk_gather / pk_scatter / pk_duplex : a kernel per relay packet (payload at
//        packet offset 12, 4-B aligned, `--stride` B apart) <-> contiguous HBM
// for hipHostMalloc'd and hipHostRegister'd (malloc'd) host memory.
// usage: hostlink [--mib M] [--size 1472] [--stride 1536] [--waves W] [--reps R]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

// Contiguous copy, 16 B per lane, grid-stride.
__global__ void k_copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// One wave per packet: payload of `size` bytes at src + p*sstride + soff (4-B
// aligned) -> dst + p*dstride + doff, dwords per lane (4 B x 64 = 256 B per
// instruction) or, when both sides are 16-B aligned, 16 B per lane.
__global__ void k_packets(const uint8_t* __restrict__ src, uint64_t sstride, uint32_t soff, uint8_t* __restrict__ dst,
                          uint64_t dstride, uint32_t doff, uint32_t size, uint64_t npk, int wide) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t p = wave; p < npk; p += nw) {
        const uint8_t* s = src + p * sstride + soff;
        uint8_t* d = dst + p * dstride + doff;
        if (wide) {
            for (uint32_t o = 16 * lane; o < size; o += 1024)
                *reinterpret_cast<uint4*>(d + o) = *reinterpret_cast<const uint4*>(s + o);
        } else {
            for (uint32_t o = 4 * lane; o < size; o += 256)
                *reinterpret_cast<uint32_t*>(d + o) = *reinterpret_cast<const uint32_t*>(s + o);
        }
    }
}

struct Host {
    uint8_t* h = nullptr;  // host address
    uint8_t* d = nullptr;  // device address of the same memory
    bool reg = false;
};

static Host host_alloc(size_t bytes, bool registered) {
    Host m;
    m.reg = registered;
    if (registered) {
        m.h = static_cast<uint8_t*>(aligned_alloc(4096, bytes));
        memset(m.h, 1, bytes);
        CK(hipHostRegister(m.h, bytes, hipHostRegisterMapped));
    } else {
        CK(hipHostMalloc(reinterpret_cast<void**>(&m.h), bytes, hipHostMallocDefault));
        memset(m.h, 1, bytes);
    }
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&m.d), m.h, 0));
    return m;
}

int main(int argc, char** argv) {
    uint64_t mib = 2048;
    uint32_t size = 1472, stride = 1536;
    int waves = 4096, reps = 5;
    for (int i = 1; i + 1 < argc; i += 2) {
        std::string a = argv[i];
        if (a == "--mib") mib = strtoull(argv[i + 1], nullptr, 10);
        else if (a == "--size") size = atoi(argv[i + 1]);
        else if (a == "--stride") stride = atoi(argv[i + 1]);
        else if (a == "--waves") waves = atoi(argv[i + 1]);
        else if (a == "--reps") reps = atoi(argv[i + 1]);
    }
    const uint64_t bytes = mib << 20;
    const uint64_t npk = bytes / stride;
    uint8_t *d0, *d1;
    CK(hipMalloc(reinterpret_cast<void**>(&d0), bytes));
    CK(hipMalloc(reinterpret_cast<void**>(&d1), bytes));
    CK(hipMemset(d0, 3, bytes));
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int threads = 256;
    const int grid = waves * 64 / threads;

    for (int registered = 0; registered < 2; registered++) {
        Host a = host_alloc(bytes, registered), b = host_alloc(bytes, registered);
        const char* kind = registered ? "hipHostRegister" : "hipHostMalloc";
        auto timed = [&](const char* name, double moved, auto&& fn) {
            fn();
            CK(hipDeviceSynchronize());
            float best = 1e30f;
            for (int r = 0; r < reps; r++) {
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0, 0));
                fn();
                CK(hipStreamSynchronize(s0));
                CK(hipStreamSynchronize(s1));
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
            }
            printf("{\"host\": \"%s\", \"pattern\": \"%s\", \"GBps\": %.2f, \"ms\": %.3f, \"bytes\": %.0f, \"waves\": %d}\n",
                   kind, name, moved / (best * 1e-3) / 1e9, best, moved, waves);
            fflush(stdout);
        };
        const uint64_t n16 = bytes / 16;
        timed("dma_h2d", bytes, [&] { CK(hipMemcpyAsync(d0, a.h, bytes, hipMemcpyHostToDevice, s0)); });
        timed("dma_d2h", bytes, [&] { CK(hipMemcpyAsync(b.h, d1, bytes, hipMemcpyDeviceToHost, s1)); });
        timed("dma_duplex", 2.0 * bytes, [&] {
            CK(hipMemcpyAsync(d0, a.h, bytes, hipMemcpyHostToDevice, s0));
            CK(hipMemcpyAsync(b.h, d1, bytes, hipMemcpyDeviceToHost, s1));
        });
        timed("k_read", bytes, [&] {
            hipLaunchKernelGGL(k_copy16, dim3(grid), dim3(threads), 0, s0, (const uint4*)a.d, (uint4*)d0, n16);
        });
        timed("k_write", bytes, [&] {
            hipLaunchKernelGGL(k_copy16, dim3(grid), dim3(threads), 0, s1, (const uint4*)d1, (uint4*)b.d, n16);
        });
        timed("k_duplex", 2.0 * bytes, [&] {
            hipLaunchKernelGGL(k_copy16, dim3(grid / 2), dim3(threads), 0, s0, (const uint4*)a.d, (uint4*)d0, n16);
            hipLaunchKernelGGL(k_copy16, dim3(grid / 2), dim3(threads), 0, s1, (const uint4*)d1, (uint4*)b.d, n16);
        });
        const double pay = (double)npk * size;
        for (int wide = 0; wide < 2; wide++) {
            // wide: 16-B aligned payloads (offset 16); narrow: the relay's offset 12 (4-B aligned)
            const uint32_t off = wide ? 16 : 12;
            const std::string sfx = wide ? "_16B" : "_4B";
            timed(("pk_gather" + sfx).c_str(), pay, [&] {
                hipLaunchKernelGGL(k_packets, dim3(grid), dim3(threads), 0, s0, a.d, (uint64_t)stride, off, d0,
                                   (uint64_t)size, 0u, size, npk, wide);
            });
            timed(("pk_scatter" + sfx).c_str(), pay, [&] {
                hipLaunchKernelGGL(k_packets, dim3(grid), dim3(threads), 0, s1, d1, (uint64_t)size, 0u, b.d,
                                   (uint64_t)stride, off, size, npk, wide);
            });
            timed(("pk_duplex" + sfx).c_str(), 2 * pay, [&] {
                hipLaunchKernelGGL(k_packets, dim3(grid / 2), dim3(threads), 0, s0, a.d, (uint64_t)stride, off, d0,
                                   (uint64_t)size, 0u, size, npk, wide);
                hipLaunchKernelGGL(k_packets, dim3(grid / 2), dim3(threads), 0, s1, d1, (uint64_t)size, 0u, b.d,
                                   (uint64_t)stride, off, size, npk, wide);
            });
        }
        // correctness spot check of the last pk_scatter (wide): packet 7's payload
        CK(hipDeviceSynchronize());
        std::vector<uint8_t> want(size);
        CK(hipMemcpy(want.data(), d1 + 7ull * size, size, hipMemcpyDeviceToHost));
        if (memcmp(want.data(), b.h + 7ull * stride + 16, size) != 0) {
            printf("{\"error\": \"scatter mismatch\"}\n");
            return 2;
        }
        if (registered) {
            CK(hipHostUnregister(a.h));
            CK(hipHostUnregister(b.h));
            free(a.h);
            free(b.h);
        } else {
            CK(hipHostFree(a.h));
            CK(hipHostFree(b.h));
        }
    }
    return 0;
}
