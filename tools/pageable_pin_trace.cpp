// tools/pageable_pin_trace.cpp -- what the HIP runtime does with a pageable
// host buffer above GPU_PINNED_MIN_XFER_SIZE during a copy, and whether
// anything of it is still held when the copy call has returned (DESIGN.md
// §4.2).  Library-free: only the HIP runtime.
//
// Run it under AMD_LOG_LEVEL=4 (the runtime's own log on stderr): each step
// prints a marker line "=== <step>" to stderr before and "--- <step> done"
// after, so the runtime's log lines fall between the markers of the call that
// produced them.  After each copy the buffer's first byte is queried
// (hipPointerGetAttributes, hipHostGetDevicePointer) and then the same live
// range is registered and unregistered once (hipHostRegister over memory that
// is mapped and owned by this program): a runtime that still held the range
// would answer the query or refuse the registration.
//
// Nothing here unmaps memory that anything may still hold or copies from
// memory that was unmapped: no step can hand the GPU a stale mapping.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

static void mark(const char* what) {
    fflush(stdout);
    fprintf(stderr, "=== %s\n", what);
    fflush(stderr);
}
static void done(const char* what, hipError_t e) {
    fprintf(stderr, "--- %s done: %s\n", what, hipGetErrorName(e));
    fflush(stderr);
    printf("%-44s -> %s\n", what, hipGetErrorName(e));
}

static void query(const char* what, void* p, size_t n) {
    hipPointerAttribute_t at = {};
    const hipError_t e1 = hipPointerGetAttributes(&at, p);
    (void)hipGetLastError();
    void* dp = nullptr;
    const hipError_t e2 = hipHostGetDevicePointer(&dp, p, 0);
    (void)hipGetLastError();
    mark("probe register (live memory)");
    const hipError_t e3 = hipHostRegister(p, n, hipHostRegisterDefault);
    (void)hipGetLastError();
    const hipError_t e4 = e3 == hipSuccess ? hipHostUnregister(p) : hipErrorUnknown;
    (void)hipGetLastError();
    done("probe register (live memory)", e3);
    printf("  %-40s attrs %s type %d | devptr %s | register %s unregister %s\n", what, hipGetErrorName(e1),
           e1 == hipSuccess ? (int)at.type : -1, hipGetErrorName(e2), hipGetErrorName(e3),
           e3 == hipSuccess ? hipGetErrorName(e4) : "-");
}

int main() {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        printf("no device\n");
        return 1;
    }
    (void)hipSetDevice(0);
    (void)hipFree(nullptr);
    const char* env = getenv("GPU_PINNED_MIN_XFER_SIZE");
    printf("GPU_PINNED_MIN_XFER_SIZE=%s\n", env ? env : "(unset: 1 MiB)");
    const size_t n = 2635124;          // the r05 fault's copy size
    const size_t region = 4u << 20;    // an mmap of its own, as numpy's allocator makes for it
    uint8_t* host = (uint8_t*)mmap(nullptr, region, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (host == MAP_FAILED) return 1;
    memset(host, 0x5a, region);
    uint8_t* src = host + 16;          // numpy's data pointer: 16 B past the mapping's start
    void* d = nullptr;
    if (hipMalloc(&d, region) != hipSuccess) return 1;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;

    query("before any copy", src, n);

    mark("hipMemcpy H2D (synchronous)");
    hipError_t e = hipMemcpy(d, src, n, hipMemcpyHostToDevice);
    done("hipMemcpy H2D (synchronous)", e);
    query("after hipMemcpy H2D", src, n);

    mark("hipMemcpyWithStream H2D (torch's pageable .to(cuda))");
    e = hipMemcpyWithStream(d, src, n, hipMemcpyHostToDevice, s);
    done("hipMemcpyWithStream H2D (torch's pageable .to(cuda))", e);
    query("after hipMemcpyWithStream H2D", src, n);

    mark("hipMemcpyAsync H2D");
    e = hipMemcpyAsync(d, src, n, hipMemcpyHostToDevice, s);
    done("hipMemcpyAsync H2D", e);
    query("after hipMemcpyAsync H2D (not synchronised)", src, n);
    mark("hipStreamSynchronize");
    e = hipStreamSynchronize(s);
    done("hipStreamSynchronize", e);
    query("after hipStreamSynchronize", src, n);

    mark("hipMemcpyWithStream D2H (torch's .cpu())");
    e = hipMemcpyWithStream(src, d, n, hipMemcpyDeviceToHost, s);
    done("hipMemcpyWithStream D2H (torch's .cpu())", e);
    query("after hipMemcpyWithStream D2H", src, n);

    mark("hipDeviceSynchronize");
    e = hipDeviceSynchronize();
    done("hipDeviceSynchronize", e);
    query("after hipDeviceSynchronize", src, n);

    (void)hipStreamDestroy(s);
    (void)hipFree(d);
    munmap(host, region);  // nothing copies from or registers this range again
    printf("done\n");
    return 0;
}
