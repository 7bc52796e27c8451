// cyaes_mgpu.cpp -- single-process multi-GPU front end (include/cyaes_mgpu.h).
// One cyaes_gpu per device; RCCL (ncclCommInitAll clique) broadcasts the raw
// session keys over xGMI; each device expands the slice its shard needs.
// Reference: SURVEY.md §8(e) -- relay payloads are independent chains
// (relay_local.cpp:206, relay_server.cpp:472), keys come from the DH owner
// (relay_server.cpp:218-240).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <vector>

#include "cyaes_mgpu.h"

struct cyaes_mgpu {
    std::vector<int> dev;
    std::vector<cyaes_gpu*> ctx;
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> stream;
    std::vector<uint8_t*> d_raw;   // raw keys, nkeys * 16 B per device
    std::vector<int64_t> base;     // first key of the expanded table (-1: none)
    uint32_t nkeys = 0;
    uint32_t raw_cap = 0;
};

namespace {

struct DevScope {  // restores the caller's current device
    int prev = 0;
    DevScope() { (void)hipGetDevice(&prev); }
    ~DevScope() { (void)hipSetDevice(prev); }
};

int map_err(hipError_t e) {
    if (e == hipSuccess) return CYAES_OK;
    return (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? CYAES_ENOMEM : CYAES_EDEVICE;
}

// Makes device i's context hold keys [k0, nkeys) (payload key p / ppk - k0).
int ensure_base(cyaes_mgpu* mg, int i, uint32_t k0) {
    if (mg->base[i] == (int64_t)k0) return CYAES_OK;
    int st = cyaes_gpu_set_keys_device(mg->ctx[i], mg->d_raw[i] + 16ull * k0, mg->nkeys - k0, mg->stream[i]);
    if (st == CYAES_OK) mg->base[i] = k0;
    return st;
}

int run(cyaes_mgpu* mg, bool decrypt, const uint8_t* const* d_in, uint8_t* const* d_out, const uint64_t* n,
        const uint64_t* first, uint32_t payload_bytes, uint32_t ppk) {
    if (!mg || !d_in || !d_out || !n || (ppk && !first)) return CYAES_EINVAL;
    if (mg->nkeys == 0) return CYAES_ERANGE;
    const int nd = (int)mg->ctx.size();
    int err = CYAES_OK;
    for (int i = 0; i < nd && err == CYAES_OK; i++) {
        if (n[i] == 0) continue;
        uint32_t k0 = 0;
        if (ppk) {
            if (first[i] % ppk) return CYAES_EINVAL;
            const uint64_t kfirst = first[i] / ppk, klast = (first[i] + n[i] - 1) / ppk;
            if (klast >= mg->nkeys) return CYAES_ERANGE;
            k0 = (uint32_t)kfirst;
        }
        err = ensure_base(mg, i, k0);
        if (err == CYAES_OK)
            err = (decrypt ? cyaes_gpu_decrypt_uniform : cyaes_gpu_encrypt_uniform)(
                mg->ctx[i], d_in[i], d_out[i], n[i], payload_bytes, nullptr, ppk, nullptr, nullptr, mg->stream[i]);
    }
    for (int i = 0; i < nd; i++) {  // every launched device drains, even after an error
        const int st = cyaes_gpu_check(mg->ctx[i]);
        if (err == CYAES_OK) err = st;
    }
    return err;
}

}  // namespace

extern "C" {

int cyaes_mgpu_create(int ndev, const int* devices, cyaes_mgpu** out) {
    if (!out || ndev < 1) return CYAES_EINVAL;
    *out = nullptr;
    DevScope scope;
    auto* mg = new cyaes_mgpu();
    for (int i = 0; i < ndev; i++) mg->dev.push_back(devices ? devices[i] : i);
    int st = CYAES_OK;
    for (int i = 0; i < ndev && st == CYAES_OK; i++) {
        cyaes_gpu* c = nullptr;
        st = cyaes_gpu_create(mg->dev[i], &c);
        if (st) break;
        mg->ctx.push_back(c);
        hipStream_t s = nullptr;
        if (hipSetDevice(mg->dev[i]) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
            st = CYAES_EDEVICE;
        mg->stream.push_back(s);
        mg->d_raw.push_back(nullptr);
        mg->base.push_back(-1);
    }
    if (st == CYAES_OK) {
        mg->comm.resize(ndev);
        if (ncclCommInitAll(mg->comm.data(), ndev, mg->dev.data()) != ncclSuccess) {
            mg->comm.clear();
            st = CYAES_EDEVICE;
        }
    }
    if (st) {
        cyaes_mgpu_destroy(mg);
        return st;
    }
    *out = mg;
    return CYAES_OK;
}

int cyaes_mgpu_destroy(cyaes_mgpu* mg) {
    if (!mg) return CYAES_OK;
    DevScope scope;
    int err = CYAES_OK;
    for (ncclComm_t c : mg->comm) (void)ncclCommDestroy(c);
    for (size_t i = 0; i < mg->ctx.size(); i++) {
        (void)hipSetDevice(mg->dev[i]);
        if (i < mg->stream.size() && mg->stream[i]) (void)hipStreamDestroy(mg->stream[i]);
        if (i < mg->d_raw.size() && mg->d_raw[i]) (void)hipFree(mg->d_raw[i]);
        const int st = cyaes_gpu_destroy(mg->ctx[i]);  // a pending fault on any device is reported
        if (err == CYAES_OK) err = st;
    }
    delete mg;
    return err;
}

int cyaes_mgpu_ndev(const cyaes_mgpu* mg) { return mg ? (int)mg->ctx.size() : 0; }

cyaes_gpu* cyaes_mgpu_context(cyaes_mgpu* mg, int i) {
    return (mg && i >= 0 && i < (int)mg->ctx.size()) ? mg->ctx[i] : nullptr;
}

int cyaes_mgpu_broadcast_keys(cyaes_mgpu* mg, const uint8_t* keys, uint32_t nkeys, int root) {
    if (!mg || !keys || nkeys == 0 || root < 0 || root >= (int)mg->ctx.size()) return CYAES_EINVAL;
    DevScope scope;
    const int nd = (int)mg->ctx.size();
    if (nkeys > mg->raw_cap) {
        for (int i = 0; i < nd; i++) {
            if (hipSetDevice(mg->dev[i]) != hipSuccess) return CYAES_EDEVICE;
            if (mg->d_raw[i]) (void)hipFree(mg->d_raw[i]);
            mg->d_raw[i] = nullptr;
            hipError_t e = hipMalloc(reinterpret_cast<void**>(&mg->d_raw[i]), 16ull * nkeys);
            if (e != hipSuccess) return map_err(e);
        }
        mg->raw_cap = nkeys;
    }
    if (hipSetDevice(mg->dev[root]) != hipSuccess) return CYAES_EDEVICE;
    hipError_t e = hipMemcpyAsync(mg->d_raw[root], keys, 16ull * nkeys, hipMemcpyHostToDevice, mg->stream[root]);
    if (e == hipSuccess) e = hipStreamSynchronize(mg->stream[root]);
    if (e != hipSuccess) return map_err(e);
    // RCCL broadcast over xGMI: one call per device inside a group (single process, many GPUs).
    if (ncclGroupStart() != ncclSuccess) return CYAES_EDEVICE;
    ncclResult_t r = ncclSuccess;
    for (int i = 0; i < nd && r == ncclSuccess; i++)
        r = ncclBroadcast(mg->d_raw[root], mg->d_raw[i], 16ull * nkeys, ncclUint8, root, mg->comm[i], mg->stream[i]);
    if (ncclGroupEnd() != ncclSuccess || r != ncclSuccess) return CYAES_EDEVICE;
    mg->nkeys = nkeys;
    int st = CYAES_OK;
    for (int i = 0; i < nd; i++) {
        mg->base[i] = -1;
        const int s = ensure_base(mg, i, 0);
        if (st == CYAES_OK) st = s;
    }
    for (int i = 0; i < nd; i++) {
        (void)hipSetDevice(mg->dev[i]);
        const hipError_t w = hipStreamSynchronize(mg->stream[i]);
        if (st == CYAES_OK) st = map_err(w);
    }
    return st;
}

int cyaes_mgpu_shard(uint64_t total, int ndev, int i, uint64_t align, uint64_t* first, uint64_t* count) {
    if (!first || !count || ndev < 1 || i < 0 || i >= ndev || align == 0) return CYAES_EINVAL;
    const uint64_t units = (total + align - 1) / align;
    auto start = [&](uint64_t r) {
        const uint64_t s = (units * r / (uint64_t)ndev) * align;
        return s < total ? s : total;
    };
    *first = start((uint64_t)i);
    *count = start((uint64_t)i + 1) - *first;
    return CYAES_OK;
}

int cyaes_mgpu_encrypt_uniform(cyaes_mgpu* mg, const uint8_t* const* d_in, uint8_t* const* d_out,
                               const uint64_t* npayloads, const uint64_t* first_payload, uint32_t payload_bytes,
                               uint32_t payloads_per_key) {
    return run(mg, false, d_in, d_out, npayloads, first_payload, payload_bytes, payloads_per_key);
}

int cyaes_mgpu_decrypt_uniform(cyaes_mgpu* mg, const uint8_t* const* d_in, uint8_t* const* d_out,
                               const uint64_t* npayloads, const uint64_t* first_payload, uint32_t payload_bytes,
                               uint32_t payloads_per_key) {
    return run(mg, true, d_in, d_out, npayloads, first_payload, payload_bytes, payloads_per_key);
}

}  // extern "C"
