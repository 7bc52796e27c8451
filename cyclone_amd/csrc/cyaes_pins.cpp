// cyaes_pins.cpp -- the one place the library registers caller host memory
// with the HIP runtime (hipHostRegister): the batcher's packet pools and the
// host-batch path's pageable buffers.
//
// Why a process-wide registry (tools/hostreg_stale_probe.hip,
// profiles/r05/hostreg_stale_probe.txt):
//  * The runtime's registration records are byte ranges keyed by their start.
//    Registering the same start twice succeeds, and one unregister then drops
//    the record: the second unregister fails (hipErrorHostMemoryNotRegistered)
//    and the second registration can no longer be released.
//  * A registration whose memory is unmapped without unregistering keeps
//    answering for new memory mapped at the same address (hipPointerGetAttributes
//    reports it registered, hipHostGetDevicePointer hands out a device address),
//    so a later pageable copy from a fresh buffer there is taken as a copy from
//    registered memory -- over a mapping that no longer exists.
// So every registration the library makes goes through here: never on a page
// someone else registered, never a second one on a page the library holds for
// a host batch, batcher pools' page spans shared by reference count (pools of
// several batchers on one page) instead of registered twice, and every
// unregister's status checked and counted.  cyaes_debug_pins() reports the counters; tests/conftest.py asserts
// after every GPU test that nothing the library registered is still live.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <deque>
#include <map>
#include <mutex>
#include <vector>

#include "cyaes.h"
#include "cyaes_internal.h"

namespace cyaes {

namespace {

// One registration the library made: host bytes [lo, hi) as registered, its
// pages [plo, phi) (the driver pins and maps whole pages).
struct Reg {
    uintptr_t phi;
    uintptr_t lo, hi;
    uint32_t refs;
    bool shared;  // a batcher pool's page span (kPinShared), else a host batch's exact range (kPinExclusive)
};

struct Registry {
    std::mutex mu;
    std::map<uintptr_t, Reg> regs;  // by first page
    uint64_t live_bytes = 0;
    uint64_t registered = 0, unregistered = 0, failed_unregisters = 0, stale = 0, foreign_conflicts = 0;
    // r06: the byte ranges released, most recent first,
    // for the test harness's after-test check that the runtime answers for
    // none of them any more; and the unregisters that found some of the
    // range's pages already unmapped (a registration that outlived its memory).
    std::deque<std::pair<uintptr_t, uintptr_t>> released;
    uint64_t outlived = 0;
};
constexpr size_t kReleasedKept = 1024;

Registry& reg() {
    static Registry r;
    return r;
}

inline uintptr_t page_down(uintptr_t a) { return a & ~(uintptr_t)(kPinPage - 1); }
inline uintptr_t page_up(uintptr_t a) { return (a + kPinPage - 1) & ~(uintptr_t)(kPinPage - 1); }

// The registration holding host byte q, if one does (another owner's, when q
// is on no page of the library's): its base as hipMemGetAddressRange reports
// it, compared only with other bytes' bases.
bool foreign_at(uintptr_t q, uintptr_t* base) {
    hipDeviceptr_t rb = nullptr;
    size_t rs = 0;
    if (hipMemGetAddressRange(&rb, &rs, reinterpret_cast<hipDeviceptr_t>(q)) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    *base = (uintptr_t)rb;
    return true;
}

// Another owner's registration on any page of [plo, phi)?  Interior pages are
// checked at their first byte, the end pages at both ends (a registration that
// starts or ends inside them).
bool foreign_in(uintptr_t plo, uintptr_t phi) {
    for (uintptr_t q = plo; q < phi; q += kPinPage) {
        uintptr_t base = 0;
        const bool edge = q == plo || q + kPinPage == phi;
        if (foreign_at(q, &base) || (edge && foreign_at(q + kPinPage - 1, &base))) return true;
    }
    return false;
}

// [lo, hi) inside one other owner's registration (a registration is one
// contiguous byte range, so its first and last byte answering with one base
// is enough).
bool inside_one_foreign(uintptr_t lo, uintptr_t hi) {
    uintptr_t b0 = 0, b1 = 0;
    return foreign_at(lo, &b0) && foreign_at(hi - 1, &b1) && b0 == b1;
}

// Unregisters one library registration (mu held) and checks that the runtime
// no longer answers for its first and last byte.
int unregister_one(Registry& r, const Reg& g) {
    // Still mapped?  msync fails with ENOMEM when a page of the range is not
    // (a query: nothing is written back for anonymous memory).
    const uintptr_t plo = page_down(g.lo);
    if (msync(reinterpret_cast<void*>(plo), page_up(g.hi) - plo, MS_ASYNC) != 0 && errno == ENOMEM) r.outlived++;
    const hipError_t e = hipHostUnregister(reinterpret_cast<void*>(g.lo));
    int st = CYAES_OK;
    if (e != hipSuccess) {
        (void)hipGetLastError();
        r.failed_unregisters++;
        st = CYAES_EDEVICE;
    } else {
        r.unregistered++;
        for (uintptr_t q : {g.lo, g.hi - 1}) {
            hipPointerAttribute_t at;
            const hipError_t a = hipPointerGetAttributes(&at, reinterpret_cast<void*>(q));
            (void)hipGetLastError();
            if (a == hipSuccess && at.type == hipMemoryTypeHost) {
                r.stale++;
                st = CYAES_EDEVICE;
                break;
            }
        }
    }
    r.live_bytes -= g.hi - g.lo;
    r.released.push_front({g.lo, g.hi});
    if (r.released.size() > kReleasedKept) r.released.pop_back();
    return st;
}

int register_one(Registry& r, uintptr_t lo, uintptr_t hi, bool shared) {
    const hipError_t e = hipHostRegister(reinterpret_cast<void*>(lo), hi - lo, hipHostRegisterMapped);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation ? CYAES_ENOMEM : CYAES_EDEVICE;
    }
    r.registered++;
    r.regs[page_down(lo)] = Reg{page_up(hi), lo, hi, 1, shared};
    r.live_bytes += hi - lo;
    return CYAES_OK;
}

}  // namespace

int pin_acquire(uintptr_t lo, uintptr_t hi, PinMode mode, PinHold* h) {
    h->regs.clear();
    h->foreign = false;
    if (lo >= hi) return CYAES_EINVAL;
    const bool shared = mode == PinMode::kShared;
    const uintptr_t plo = page_down(lo), phi = page_up(hi);
    Registry& r = reg();
    std::lock_guard<std::mutex> lk(r.mu);
    // The library's registrations on pages of [plo, phi), in address order, and the page gaps between them.
    std::vector<uintptr_t> ours;
    std::vector<std::pair<uintptr_t, uintptr_t>> gaps;
    bool exclusive_hit = false;
    auto it = r.regs.upper_bound(plo);
    if (it != r.regs.begin() && std::prev(it)->second.phi > plo) --it;
    uintptr_t c = plo;
    for (; it != r.regs.end() && it->first < phi; ++it) {
        if (it->first > c) gaps.push_back({c, it->first});
        ours.push_back(it->first);
        exclusive_hit = exclusive_hit || !it->second.shared;
        c = std::max(c, it->second.phi);
    }
    if (c < phi) gaps.push_back({c, phi});
    // Memory someone else registered, used as it is: the test runs on the exact
    // bytes (a pool at the tail of a registration whose size is not
    // a page multiple lies inside it, its page span does not).
    if (ours.empty() && inside_one_foreign(lo, hi)) {
        h->foreign = true;
        return CYAES_OK;
    }
    // Never a second registration on a page the library holds for a host
    // batch, nor on a page another owner registered (the driver pins and
    // unpins whole pages); a host batch's range takes pages nobody holds.
    if (exclusive_hit || (!shared && !ours.empty())) {
        r.foreign_conflicts++;
        return kPinConflict;
    }
    for (const auto& g : gaps)
        if (foreign_in(g.first, g.second)) {
            r.foreign_conflicts++;
            return kPinConflict;
        }
    if (!shared) {  // the exact byte range: the runtime answers for no neighbour on its end pages
        const int st = register_one(r, lo, hi, false);
        if (st) return st;
        h->regs.push_back(plo);
        return CYAES_OK;
    }
    // A pool's pages: the library's shared registrations on them are shared, the gaps registered.
    std::vector<uintptr_t> added;
    for (const auto& g : gaps) {
        const int st = register_one(r, g.first, g.second, true);
        if (st) {
            for (uintptr_t a : added) {
                const Reg ga = r.regs[a];
                r.regs.erase(a);
                (void)unregister_one(r, ga);
            }
            return st;
        }
        added.push_back(g.first);
    }
    for (uintptr_t k : ours) r.regs[k].refs++;
    ours.insert(ours.end(), added.begin(), added.end());
    h->regs = std::move(ours);
    return CYAES_OK;
}

int pin_release(PinHold* h) {
    int st = CYAES_OK;
    if (!h->regs.empty()) {
        Registry& r = reg();
        std::lock_guard<std::mutex> lk(r.mu);
        for (uintptr_t k : h->regs) {
            auto it = r.regs.find(k);
            if (it == r.regs.end()) {  // (cannot happen: a held reference keeps the entry)
                st = CYAES_EDEVICE;
                continue;
            }
            if (--it->second.refs) continue;
            const Reg g = it->second;
            r.regs.erase(it);
            const int s = unregister_one(r, g);
            if (st == CYAES_OK) st = s;
        }
    }
    h->regs.clear();
    h->foreign = false;
    return st;
}

void pin_bounds(const PinHold& h, std::vector<uintptr_t>* out) {
    Registry& r = reg();
    std::lock_guard<std::mutex> lk(r.mu);
    for (uintptr_t k : h.regs) {
        auto it = r.regs.find(k);
        if (it == r.regs.end()) continue;
        out->push_back(it->second.lo);
        out->push_back(it->second.hi);
    }
}

}  // namespace cyaes

extern "C" int cyaes_debug_pins(uint64_t out[8]) {
    if (!out) return CYAES_EINVAL;
    cyaes::Registry& r = cyaes::reg();
    std::lock_guard<std::mutex> lk(r.mu);
    out[0] = r.regs.size();
    out[1] = r.live_bytes;
    out[2] = r.registered;
    out[3] = r.unregistered;
    out[4] = r.failed_unregisters;
    out[5] = r.stale;
    out[6] = r.foreign_conflicts;
    uint64_t refs = 0;
    for (const auto& kv : r.regs) refs += kv.second.refs;
    out[7] = refs;
    return CYAES_OK;
}

extern "C" uint64_t cyaes_debug_pin_history(uint64_t* out, uint64_t cap, uint64_t* outlived) {
    cyaes::Registry& r = cyaes::reg();
    std::lock_guard<std::mutex> lk(r.mu);
    if (outlived) *outlived = r.outlived;
    uint64_t n = 0;
    for (const auto& x : r.released) {
        if (!out || n == cap) break;
        out[2 * n] = x.first;
        out[2 * n + 1] = x.second;
        n++;
    }
    return n;
}
