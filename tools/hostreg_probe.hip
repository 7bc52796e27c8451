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

int main() {
    uint8_t* m = (uint8_t*)aligned_alloc(4096, 16 * 4096);
    uint8_t* P = m;  // page 0
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
