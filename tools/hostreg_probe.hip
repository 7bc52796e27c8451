// tools/hostreg_probe.hip -- how the HIP runtime answers hipMemGetAddressRange
// for host memory registered with hipHostRegister (the batcher's pool checks,
// cyaes_batcher.cpp pin_span): adjacent and nested registrations, before and
// after unregistering a neighbour.  Prints one line per query.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static void q(const char* what, uint8_t* base, uint8_t* p) {
    hipDeviceptr_t rb = nullptr;
    size_t rs = 0;
    hipError_t e = hipMemGetAddressRange(&rb, &rs, (hipDeviceptr_t)p);
    (void)hipGetLastError();
    if (e == hipSuccess)
        printf("%-34s page %+.2f -> [%+.2f, %+.2f) pages\n", what, (p - base) / 4096.0, ((uint8_t*)rb - base) / 4096.0,
               ((uint8_t*)rb + rs - base) / 4096.0);
    else
        printf("%-34s page %+.2f -> %s\n", what, (p - base) / 4096.0, hipGetErrorName(e));
}

// The addresses each query returns for host page q of a registration: the
// host pointer, hipHostGetDevicePointer, hipMemGetAddressRange's base, and
// hipPointerGetAttributes' device and host pointers (relative to q, in bytes).
static void addrs(const char* what, uint8_t* q) {
    void* dq = nullptr;
    hipDeviceptr_t rb = nullptr;
    size_t rs = 0;
    hipPointerAttribute_t at = {};
    const hipError_t e1 = hipHostGetDevicePointer(&dq, q, 0);
    const hipError_t e2 = hipMemGetAddressRange(&rb, &rs, (hipDeviceptr_t)q);
    const hipError_t e3 = hipPointerGetAttributes(&at, q);
    (void)hipGetLastError();
    printf("%-24s devptr %s %+lld | range %s base %+lld size %zu | attrs %s type %d dev %+lld host %+lld\n", what,
           hipGetErrorName(e1), (long long)((uint8_t*)dq - q), hipGetErrorName(e2), (long long)((uint8_t*)rb - q), rs,
           hipGetErrorName(e3), (int)at.type, (long long)((uint8_t*)at.devicePointer - q),
           (long long)((uint8_t*)at.hostPointer - q));
}

int main() {
    uint8_t* m = (uint8_t*)aligned_alloc(4096, 16 * 4096);
    uint8_t* P = m;  // page 0
    {  // flags 0 (what torch's cudaHostRegister passes) and mapped, queried at the start and inside
        uint8_t* a = P + 8 * 4096;
        printf("register [8,12) flags 0: %s\n", hipGetErrorName(hipHostRegister(a, 4 * 4096, 0)));
        addrs("flags0 page 8", a);
        addrs("flags0 page 9 + 100", a + 4096 + 100);
        (void)hipHostUnregister(a);
        printf("register [8,12) mapped: %s\n", hipGetErrorName(hipHostRegister(a, 4 * 4096, hipHostRegisterMapped)));
        addrs("mapped page 8", a);
        addrs("mapped page 9 + 100", a + 4096 + 100);
        (void)hipHostUnregister(a);
        (void)hipGetLastError();
    }
    printf("register [1,5): %s\n", hipGetErrorName(hipHostRegister(P + 4096, 4 * 4096, hipHostRegisterMapped)));
    for (int i = 0; i <= 6; i++) q("after [1,5)", P, P + i * 4096 + (i == 2 ? 100 : 0));
    printf("register [5,7): %s\n", hipGetErrorName(hipHostRegister(P + 5 * 4096, 2 * 4096, hipHostRegisterMapped)));
    for (int i = 0; i <= 7; i++) q("after [5,7)", P, P + i * 4096);
    void* d1 = nullptr;
    void* d2 = nullptr;
    (void)hipHostGetDevicePointer(&d1, P + 4 * 4096, 0);
    (void)hipHostGetDevicePointer(&d2, P + 5 * 4096, 0);
    printf("device ptr delta page4->page5: %lld (host 4096)\n", (long long)((uint8_t*)d2 - (uint8_t*)d1));
    printf("unregister [5,7): %s\n", hipGetErrorName(hipHostUnregister(P + 5 * 4096)));
    for (int i = 0; i <= 7; i++) q("after unregister [5,7)", P, P + i * 4096);
    printf("register [0,3) over [1,5): %s\n", hipGetErrorName(hipHostRegister(P, 3 * 4096, hipHostRegisterMapped)));
    (void)hipGetLastError();
    printf("unregister [1,5): %s\n", hipGetErrorName(hipHostUnregister(P + 4096)));
    (void)hipGetLastError();
    for (int i = 0; i <= 5; i++) q("end", P, P + i * 4096);
    printf("unregister [0,3): %s\n", hipGetErrorName(hipHostUnregister(P)));
    return 0;
}
