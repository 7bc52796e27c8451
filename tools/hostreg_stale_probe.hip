// tools/hostreg_stale_probe.hip -- what the HIP runtime believes about host
// pages around hipHostRegister / hipHostUnregister, for the r04
// illegal-address reports.  Host-side queries, and copies
// only between hipMalloc memory and live, unregistered pageable memory (the
// ordinary pageable path): nothing here hands the GPU a stale mapping.
//
// For each scenario it prints, per probed address, whether
// hipPointerGetAttributes calls it registered host memory and whether
// hipHostGetDevicePointer hands out a device address for it, plus the status
// of every register / unregister.  Scenarios:
//   end      the first byte after a registration (page-aligned and unaligned)
//   shared   HostPin's in/out pattern: two ranges sharing one page, in that
//            order registered, unregistered in either order
//   overlap  two page-aligned registrations with different starts overlapping
//   twice    the same range registered twice
//   pageable whether a pageable copy above 1 MiB leaves its pages locked
//   leak     (only with argument "leak") a registration whose memory is
//            unmapped without unregistering, then new memory mapped at the
//            same address: is the old record still answered for it?
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

static const size_t PG = 4096;

static const char* st(hipError_t e) { return hipGetErrorName(e); }

static void q(const char* what, const uint8_t* base, const uint8_t* p) {
    hipPointerAttribute_t at = {};
    const hipError_t e1 = hipPointerGetAttributes(&at, p);
    (void)hipGetLastError();
    void* dp = nullptr;
    const hipError_t e2 = hipHostGetDevicePointer(&dp, const_cast<uint8_t*>(p), 0);
    (void)hipGetLastError();
    // ROCr's own view (the layer a pageable copy above 1 MiB pins through)
    hsa_amd_pointer_info_t pi = {};
    pi.size = sizeof(pi);
    const hsa_status_t e3 = hsa_amd_pointer_info(const_cast<uint8_t*>(p), &pi, nullptr, nullptr, nullptr);
    printf("  %-28s @page %+8.4f  hip: attrs %-11s type %2d devptr %-22s | rocr: %d type %d host %+.4f size %.4f agent-host %+lld\n",
           what, (p - base) / 4096.0, e1 == hipSuccess ? "ok" : st(e1), e1 == hipSuccess ? (int)at.type : -1, st(e2),
           (int)e3, (int)pi.type, pi.type ? ((const uint8_t*)pi.hostBaseAddress - base) / 4096.0 : 0.0,
           pi.type ? pi.sizeInBytes / 4096.0 : 0.0,
           pi.type ? (long long)((uint8_t*)pi.agentBaseAddress - (uint8_t*)pi.hostBaseAddress) : 0LL);
}

static hipError_t reg(const char* what, void* p, size_t n) {
    const hipError_t e = hipHostRegister(p, n, hipHostRegisterDefault);
    (void)hipGetLastError();
    printf("register   %-22s -> %s\n", what, st(e));
    return e;
}

static hipError_t unreg(const char* what, void* p) {
    const hipError_t e = hipHostUnregister(p);
    (void)hipGetLastError();
    printf("unregister %-22s -> %s\n", what, st(e));
    return e;
}

static uint8_t* fresh(size_t pages) {
    void* m = mmap(nullptr, pages * PG, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) {
        perror("mmap");
        exit(1);
    }
    memset(m, 1, pages * PG);
    return (uint8_t*)m;
}

int main(int argc, char** argv) {
    const bool leak = argc > 1 && !strcmp(argv[1], "leak");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        printf("no device\n");
        return 1;
    }
    (void)hipSetDevice(0);
    (void)hipFree(nullptr);
    (void)hsa_init();  // refcounted: the HIP runtime already holds one

    {
        printf("== end: [1,5) page-aligned\n");
        uint8_t* P = fresh(8);
        reg("[1,5)", P + PG, 4 * PG);
        q("page 1", P, P + PG);
        q("last byte (5 - 1B)", P, P + 5 * PG - 1);
        q("first byte after (5)", P, P + 5 * PG);
        q("5 + 16", P, P + 5 * PG + 16);
        q("before (1 - 1B)", P, P + PG - 1);
        unreg("[1,5)", P + PG);
        q("page 1 after", P, P + PG);
        q("5 after", P, P + 5 * PG);
        munmap(P, 8 * PG);
    }
    {
        printf("== end: unaligned [1+16, 4+16)\n");
        uint8_t* P = fresh(8);
        uint8_t* A = P + PG + 16;
        reg("[1+16, 4+16)", A, 3 * PG);
        q("page 1 start (before A)", P, P + PG);
        q("A", P, A);
        q("last byte", P, A + 3 * PG - 1);
        q("first byte after", P, A + 3 * PG);
        q("first byte after + 16", P, A + 3 * PG + 16);
        q("page 5 start", P, P + 5 * PG);
        unreg("A", A);
        q("A after", P, A);
        q("first byte after, after", P, A + 3 * PG);
        munmap(P, 8 * PG);
    }
    for (int order = 0; order < 2; order++) {
        printf("== shared: in [1+16, 3+16), out [3+32, 5+32), unregister %s first\n", order ? "in" : "out");
        uint8_t* P = fresh(8);
        uint8_t* in = P + PG + 16;
        uint8_t* out = P + 3 * PG + 32;
        reg("in", in, 2 * PG);
        q("out before its register", P, out);
        reg("out", out, 2 * PG);
        q("in", P, in);
        q("out", P, out);
        q("shared page start", P, P + 3 * PG);
        if (order) {
            unreg("in", in);
            q("in after in", P, in);
            q("out after in", P, out);
            unreg("out", out);
        } else {
            unreg("out", out);
            q("in after out", P, in);
            q("out after out", P, out);
            unreg("in", in);
        }
        for (int i = 0; i <= 6; i++) q("end: page", P, P + i * PG + 40);
        munmap(P, 8 * PG);
    }
    {
        printf("== overlap: [0,3) then [2,6)\n");
        uint8_t* P = fresh(8);
        reg("[0,3)", P, 3 * PG);
        reg("[2,6) over it", P + 2 * PG, 4 * PG);
        for (int i = 0; i <= 6; i++) q("both: page", P, P + i * PG);
        unreg("[0,3)", P);
        for (int i = 0; i <= 6; i++) q("after [0,3): page", P, P + i * PG);
        unreg("[2,6)", P + 2 * PG);
        for (int i = 0; i <= 6; i++) q("end: page", P, P + i * PG);
        munmap(P, 8 * PG);
    }
    {
        printf("== twice: [1,3) registered twice\n");
        uint8_t* P = fresh(4);
        reg("[1,3)", P + PG, 2 * PG);
        reg("[1,3) again", P + PG, 2 * PG);
        unreg("[1,3)", P + PG);
        q("after one unregister", P, P + PG);
        unreg("[1,3) again", P + PG);
        q("after two", P, P + PG);
        munmap(P, 4 * PG);
    }
    {
        printf("== pageable: 2 MiB H2D and D2H from and to fresh pageable memory (no registration)\n");
        uint8_t* P = fresh(1024);
        void* d = nullptr;
        if (hipMalloc(&d, 4 << 20) != hipSuccess) return 1;
        q("before copy", P, P);
        printf("hipMemcpy H2D 2 MiB -> %s\n", st(hipMemcpy(d, P, 2 << 20, hipMemcpyHostToDevice)));
        printf("sync -> %s\n", st(hipDeviceSynchronize()));
        q("after H2D: page 0", P, P);
        q("after H2D: page 300", P, P + 300 * PG);
        printf("hipMemcpy D2H 2 MiB -> %s\n", st(hipMemcpy(P + 2048 * 1024, d, 2 << 20, hipMemcpyDeviceToHost)));
        q("after D2H: page 512", P, P + 512 * PG);
        printf("hipMemcpy H2D 512 KiB -> %s\n", st(hipMemcpy(d, P, 512 << 10, hipMemcpyHostToDevice)));
        q("after small H2D: page 0", P, P);
        (void)hipFree(d);
        munmap(P, 1024 * PG);
    }
    if (leak) {
        printf("== leak: [0,4) registered, unmapped without unregister, new memory at the same address\n");
        uint8_t* P = fresh(4);
        reg("[0,4)", P, 4 * PG);
        munmap(P, 4 * PG);
        void* m = mmap(P, 4 * PG, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED_NOREPLACE, -1, 0);
        if (m != P) {
            printf("  remap at the same address failed (%p)\n", m);
        } else {
            memset(P, 2, 4 * PG);
            q("new memory, page 0", P, P);
            q("new memory, page 2 + 100", P, P + 2 * PG + 100);
            unreg("stale [0,4)", P);
            q("after unregister", P, P);
            munmap(P, 4 * PG);
        }
    }
    printf("done\n");
    return 0;
}
