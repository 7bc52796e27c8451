// cyaes_batcher.cpp -- asynchronous batching adapter (include/cyaes_batch.h).
//
// Reference call pattern being replaced: synchronous per-packet
// Rijndael::encrypt / decrypt on the looper threads of samples/relay
// (relay_local.cpp:188-217, 365; relay_server.cpp:329, 453-481), with one
// Rijndael pair per pipe created after the DH handshake
// (relay_server.cpp:218-240) and deleted on close (:370-375).
//
// Threads: callers submit into a queue; the builder thread closes a batch
// when it is full, when its oldest request has waited max_delay_us, or when
// someone flushes, gathers it into a pinned staging buffer and launches
// H2D -> ragged encrypt -> ragged decrypt -> D2H on that stage's stream; the
// completion thread waits for the stage, scatters outputs, runs callbacks and
// recycles the stage.  Staging layout of one batch (one H2D, one D2H):
//   [data: each request 16-B aligned][enc meta][dec meta][key schedules]
// A SEAL/OPEN request keeps its packet at data offset o + 4 so the payload
// (packet offset 12) sits at o + 16.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "cyaes.h"
#include "cyaes_batch.h"
#include "cyaes_internal.h"
#include "cyaes_relay.h"
#include "cyaes_tables.h"

namespace {

using Clock = std::chrono::steady_clock;
using Sched = std::array<uint32_t, cyaes::kSchedWords>;  // device-format schedule (cyaes_internal.h)

uint64_t up16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

struct Req {
    uint8_t op;
    std::shared_ptr<const Sched> key;  // pinned at submit: a later close/reopen does not affect it
    const uint8_t* in;
    uint8_t* out;
    uint32_t size;      // ENC/DEC: bytes; SEAL: chunk bytes; OPEN: packet bytes
    uint32_t crypt;     // bytes the kernel processes
    int32_t conn;       // SEAL: RelayForwardMsg::id
    cyaes_done_fn done;
    void* user;
    Clock::time_point t;
    uint64_t data_bytes() const { return up16(op >= CYAES_OP_RELAY_SEAL ? 16 + crypt : size); }
};

struct Stage {
    uint8_t* h = nullptr;  // pinned
    uint8_t* d = nullptr;  // device
    uint64_t cap = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    std::vector<Req> reqs;
    std::vector<uint64_t> off;  // data offset per request
    uint64_t data_end = 0;
    int status = CYAES_OK;
};

int map_err(hipError_t e) {
    if (e == hipSuccess) return CYAES_OK;
    return (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? CYAES_ENOMEM : CYAES_EDEVICE;
}

}  // namespace

struct cyaes_batcher {
    cyaes_batcher_config cfg{};
    cyaes_gpu* ctx = nullptr;
    uint64_t stage_cap = 0;
    std::vector<Stage> stages;

    std::mutex mu;
    std::condition_variable cv_submit, cv_free, cv_inflight, cv_flush;
    std::deque<Req> queue;
    uint64_t queued_bytes = 0;
    std::vector<Stage*> free_stages;
    std::deque<Stage*> inflight;
    bool stop = false, builder_done = false;
    int flushers = 0;
    uint64_t submitted = 0, completed = 0;
    uint64_t batches = 0, bytes = 0, max_batch = 0, errors = 0;
    int first_error = CYAES_OK;

    std::vector<std::shared_ptr<const Sched>> sessions;  // nullptr = free slot

    std::thread builder, completer;

    // Cost of a request in a stage: data + meta (16 B) + a schedule if its key is new to the batch.
    static uint64_t cost(const Req& r) { return r.data_bytes() + 16; }

    void build_loop();
    void complete_loop();
    int launch(Stage* st);
    int submit(Req&& r);
};

void cyaes_batcher::build_loop() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
        cv_submit.wait(lk, [&] { return stop || !queue.empty(); });
        if (queue.empty()) break;  // stop requested and drained
        // Let the batch fill: until it is full, the oldest request is due, or a flush/stop.
        const auto due = queue.front().t + std::chrono::microseconds(cfg.max_delay_us);
        cv_submit.wait_until(lk, due, [&] { return stop || flushers > 0 || queued_bytes >= cfg.max_batch_bytes; });
        cv_free.wait(lk, [&] { return !free_stages.empty(); });
        Stage* st = free_stages.back();
        free_stages.pop_back();
        st->reqs.clear();
        uint64_t used = 0, data = 0;
        std::unordered_map<const Sched*, int> seen;
        while (!queue.empty()) {
            const Req& r = queue.front();
            const bool new_key = !seen.count(r.key.get());
            const uint64_t c = cost(r) + (new_key ? sizeof(Sched) : 0);
            if (!st->reqs.empty() && (data + r.data_bytes() > cfg.max_batch_bytes || used + c + 64 > stage_cap))
                break;
            if (new_key) seen.emplace(r.key.get(), 0);
            used += c;
            data += r.data_bytes();
            queued_bytes -= r.data_bytes();
            st->reqs.push_back(std::move(queue.front()));
            queue.pop_front();
        }
        lk.unlock();
        st->status = launch(st);
        lk.lock();
        inflight.push_back(st);
        cv_inflight.notify_one();
    }
    builder_done = true;
    cv_inflight.notify_all();
}

// Gathers st->reqs into the stage and launches the batch on its stream.
int cyaes_batcher::launch(Stage* st) {
    const size_t n = st->reqs.size();
    st->off.resize(n);
    // Data section + per-direction lists.
    std::vector<uint64_t> eo, doff;
    std::vector<uint32_t> el, ek, dl, dk;
    std::unordered_map<const Sched*, uint32_t> kidx;
    std::vector<const Sched*> klist;
    uint64_t pos = 0;
    for (size_t i = 0; i < n; i++) {
        const Req& r = st->reqs[i];
        st->off[i] = pos;
        uint8_t* dst = st->h + pos;
        uint64_t coff = pos;  // where the kernel works
        switch (r.op) {
            case CYAES_OP_ENCRYPT:
            case CYAES_OP_DECRYPT:
                memcpy(dst, r.in, r.size);
                break;
            case CYAES_OP_RELAY_SEAL:  // relay_local.cpp:189-201: packet build + 0xCE padding
                cyaes_relay_build_forward(dst + 4, r.conn, r.in, r.size);
                coff = pos + 16;
                break;
            case CYAES_OP_RELAY_OPEN:
                memcpy(dst + 4, r.in, r.size);
                coff = pos + 16;
                break;
        }
        pos += r.data_bytes();
        if (r.crypt == 0) continue;  // size 0: a no-op (cyr_rijndael.cpp:600 loop never runs)
        auto it = kidx.find(r.key.get());
        uint32_t k;
        if (it == kidx.end()) {
            k = (uint32_t)klist.size();
            kidx.emplace(r.key.get(), k);
            klist.push_back(r.key.get());
        } else {
            k = it->second;
        }
        const bool dec = r.op == CYAES_OP_DECRYPT || r.op == CYAES_OP_RELAY_OPEN;
        (dec ? doff : eo).push_back(coff);
        (dec ? dl : el).push_back(r.crypt);
        (dec ? dk : ek).push_back(k);
    }
    st->data_end = pos;
    // Encrypt runs one chain per lane and waterfalls over the distinct keys of
    // a wave (cyaes_kernels.hip, k_encrypt), so order its list by key: a wave
    // then sees one key, two at a boundary, instead of one per looper thread.
    // (Decrypt runs one payload per wave: one key per wave already.)
    if (klist.size() > 1 && !eo.empty()) {
        std::vector<uint32_t> ord(eo.size());
        for (uint32_t i = 0; i < ord.size(); i++) ord[i] = i;
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return ek[x] < ek[y]; });
        std::vector<uint64_t> o2(eo.size());
        std::vector<uint32_t> l2(el.size()), k2(ek.size());
        for (size_t i = 0; i < ord.size(); i++) o2[i] = eo[ord[i]], l2[i] = el[ord[i]], k2[i] = ek[ord[i]];
        // Small batch: start every key group on a wave boundary with empty
        // (0-byte) lanes, so no wave waterfalls; the waves are then all
        // latency-bound chains on separate CUs (A/B on bench_batcher seal 1472 B).
        uint64_t waves = 0;
        for (size_t i = 0; i < k2.size();) {
            size_t j = i;
            while (j < k2.size() && k2[j] == k2[i]) j++;
            waves += (j - i + 63) / 64;
            i = j;
        }
        if (waves <= 4096) {
            eo.clear(), el.clear(), ek.clear();
            for (size_t i = 0; i < k2.size(); i++) {
                if (i && k2[i] != k2[i - 1])
                    while (eo.size() % 64) eo.push_back(0), el.push_back(0), ek.push_back(k2[i - 1]);
                eo.push_back(o2[i]), el.push_back(l2[i]), ek.push_back(k2[i]);
            }
        } else {
            eo.swap(o2);
            el.swap(l2);
            ek.swap(k2);
        }
    }
    // Meta + keys after the data.
    auto put = [&](const void* src, size_t bytes) {
        const uint64_t at = pos;
        if (bytes) memcpy(st->h + at, src, bytes);
        pos = up16(pos + bytes);
        return at;
    };
    const uint64_t eo_at = put(eo.data(), eo.size() * 8), el_at = put(el.data(), el.size() * 4),
                   ek_at = put(ek.data(), ek.size() * 4);
    const uint64_t do_at = put(doff.data(), doff.size() * 8), dl_at = put(dl.data(), dl.size() * 4),
                   dk_at = put(dk.data(), dk.size() * 4);
    const uint64_t keys_at = pos;
    for (const Sched* s : klist) put(s->data(), sizeof(Sched));
    if (pos > st->cap) return CYAES_ENOMEM;  // cannot happen: cost() bounds it

    hipError_t e = hipMemcpyAsync(st->d, st->h, pos, hipMemcpyHostToDevice, st->stream);
    if (e != hipSuccess) return map_err(e);
    const uint32_t* table = reinterpret_cast<const uint32_t*>(st->d + keys_at);
    const uint32_t nk = (uint32_t)klist.size();
    int rc = CYAES_OK;
    if (!eo.empty())
        rc = cyaes::ragged_batch(ctx, false, table, nk, st->d, st->d, reinterpret_cast<const uint64_t*>(st->d + eo_at),
                                 reinterpret_cast<const uint32_t*>(st->d + el_at), eo.size(),
                                 reinterpret_cast<const uint32_t*>(st->d + ek_at), st->stream);
    if (rc == CYAES_OK && !doff.empty())
        rc = cyaes::ragged_batch(ctx, true, table, nk, st->d, st->d, reinterpret_cast<const uint64_t*>(st->d + do_at),
                                 reinterpret_cast<const uint32_t*>(st->d + dl_at), doff.size(),
                                 reinterpret_cast<const uint32_t*>(st->d + dk_at), st->stream);
    if (rc != CYAES_OK) return rc;
    e = hipMemcpyAsync(st->h, st->d, st->data_end, hipMemcpyDeviceToHost, st->stream);
    if (e == hipSuccess) e = hipEventRecord(st->done, st->stream);
    return map_err(e);
}

void cyaes_batcher::complete_loop() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
        cv_inflight.wait(lk, [&] { return !inflight.empty() || builder_done; });
        if (inflight.empty()) break;
        Stage* st = inflight.front();
        inflight.pop_front();
        lk.unlock();
        int status = st->status;
        if (status == CYAES_OK) status = map_err(hipEventSynchronize(st->done));
        uint64_t nbytes = 0;
        for (size_t i = 0; i < st->reqs.size(); i++) {
            const Req& r = st->reqs[i];
            const uint8_t* src = st->h + st->off[i];
            if (status == CYAES_OK) {
                switch (r.op) {
                    case CYAES_OP_ENCRYPT:
                    case CYAES_OP_DECRYPT:
                        memcpy(r.out, src, r.size);
                        break;
                    case CYAES_OP_RELAY_SEAL:
                        memcpy(r.out, src + 4, CYAES_RELAY_PAYLOAD_OFFSET + r.crypt);
                        break;
                    case CYAES_OP_RELAY_OPEN:  // header untouched, payload decrypted in place
                        memcpy(r.out + CYAES_RELAY_PAYLOAD_OFFSET, src + 16, r.crypt);
                        break;
                }
            }
            nbytes += r.crypt;
            if (r.done) r.done(r.user, status);
        }
        const size_t nreq = st->reqs.size();
        st->reqs.clear();  // drops the schedule references
        lk.lock();
        completed += nreq;
        batches++;
        bytes += nbytes;
        max_batch = std::max<uint64_t>(max_batch, nreq);
        if (status != CYAES_OK) {
            errors += nreq;
            if (first_error == CYAES_OK) first_error = status;
        }
        free_stages.push_back(st);
        cv_free.notify_one();
        cv_flush.notify_all();
    }
}

int cyaes_batcher::submit(Req&& r) {
    r.t = Clock::now();
    std::lock_guard<std::mutex> lk(mu);
    if (stop) return CYAES_EINVAL;
    queued_bytes += r.data_bytes();
    submitted++;
    queue.push_back(std::move(r));
    if (queue.size() == 1 || queued_bytes >= cfg.max_batch_bytes) cv_submit.notify_one();
    return CYAES_OK;
}

extern "C" {

int cyaes_batcher_create(const cyaes_batcher_config* cfg, cyaes_batcher** out) {
    if (!cfg || !out) return CYAES_EINVAL;
    *out = nullptr;
    cyaes_batcher_config c = *cfg;
    if (c.max_batch_bytes == 0) c.max_batch_bytes = 32u << 20;
    if (c.max_delay_us == 0) c.max_delay_us = 100;
    if (c.inflight == 0) c.inflight = 3;
    if (c.max_batch_bytes < 4096 || c.max_batch_bytes > (1u << 30) || c.inflight > 16) return CYAES_EINVAL;
    cyaes_gpu* ctx = nullptr;
    int st = cyaes_gpu_create(c.device, &ctx);
    if (st) return st;
    auto* b = new cyaes_batcher();
    b->cfg = c;
    b->ctx = ctx;
    // A stage holds max_batch_bytes of data plus meta and schedules: cost() is at
    // most (data + 16 + 352) per request, and data >= 16 unless the request is empty.
    b->stage_cap = 2ull * c.max_batch_bytes + 64 * 1024;
    b->stages.resize(c.inflight);
    int dev_prev = 0;
    (void)hipGetDevice(&dev_prev);
    hipError_t e = hipSetDevice(c.device);
    for (Stage& s : b->stages) {
        if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&s.h), b->stage_cap, hipHostMallocDefault);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s.d), b->stage_cap);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
        s.cap = b->stage_cap;
        b->free_stages.push_back(&s);
    }
    (void)hipSetDevice(dev_prev);
    if (e != hipSuccess) {
        b->builder_done = true;
        cyaes_batcher_destroy(b);
        return map_err(e);
    }
    b->builder = std::thread([b] {
        (void)hipSetDevice(b->cfg.device);
        b->build_loop();
    });
    b->completer = std::thread([b] {
        (void)hipSetDevice(b->cfg.device);
        b->complete_loop();
    });
    *out = b;
    return CYAES_OK;
}

void cyaes_batcher_destroy(cyaes_batcher* b) {
    if (!b) return;
    {
        std::lock_guard<std::mutex> lk(b->mu);
        b->stop = true;
    }
    b->cv_submit.notify_all();
    if (b->builder.joinable()) b->builder.join();
    if (b->completer.joinable()) b->completer.join();
    for (Stage& s : b->stages) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.stream) (void)hipStreamDestroy(s.stream);
        if (s.d) (void)hipFree(s.d);
        if (s.h) (void)hipHostFree(s.h);
    }
    cyaes_gpu_destroy(b->ctx);
    delete b;
}

int cyaes_batcher_session_open(cyaes_batcher* b, const uint8_t key[16], uint32_t* slot) {
    if (!b || !key || !slot) return CYAES_EINVAL;
    cyaes_key k;
    cyaes::expand_key(key, &k);
    auto s = std::make_shared<Sched>();
    cyaes::to_device_schedule(k, s->data());
    std::lock_guard<std::mutex> lk(b->mu);
    size_t i = 0;
    while (i < b->sessions.size() && b->sessions[i]) i++;
    if (i == b->sessions.size()) b->sessions.emplace_back();
    b->sessions[i] = std::move(s);
    *slot = (uint32_t)i;
    return CYAES_OK;
}

int cyaes_batcher_session_close(cyaes_batcher* b, uint32_t slot) {
    if (!b) return CYAES_EINVAL;
    std::lock_guard<std::mutex> lk(b->mu);
    if (slot >= b->sessions.size() || !b->sessions[slot]) return CYAES_ERANGE;
    b->sessions[slot].reset();
    return CYAES_OK;
}

static int session_key(cyaes_batcher* b, uint32_t slot, std::shared_ptr<const Sched>* key) {
    std::lock_guard<std::mutex> lk(b->mu);
    if (slot >= b->sessions.size() || !b->sessions[slot]) return CYAES_ERANGE;
    *key = b->sessions[slot];
    return CYAES_OK;
}

int cyaes_batcher_submit(cyaes_batcher* b, int op, uint32_t slot, const uint8_t* in, uint8_t* out, size_t size,
                         cyaes_done_fn done, void* user) {
    if (!b || (op != CYAES_OP_ENCRYPT && op != CYAES_OP_DECRYPT) || size % 16 || size > b->cfg.max_batch_bytes ||
        (size && (!in || !out)))
        return CYAES_EINVAL;
    Req r{};
    int st = session_key(b, slot, &r.key);
    if (st) return st;
    r.op = (uint8_t)op;
    r.in = in;
    r.out = out;
    r.size = r.crypt = (uint32_t)size;
    r.done = done;
    r.user = user;
    return b->submit(std::move(r));
}

int cyaes_batcher_submit_seal(cyaes_batcher* b, uint32_t slot, int32_t conn_id, const uint8_t* payload,
                              uint32_t size, uint8_t* packet_out, cyaes_done_fn done, void* user) {
    if (!b || !packet_out || size > CYAES_RELAY_MAX_CHUNK || (size && !payload)) return CYAES_EINVAL;
    Req r{};
    int st = session_key(b, slot, &r.key);
    if (st) return st;
    r.op = CYAES_OP_RELAY_SEAL;
    r.in = payload;
    r.out = packet_out;
    r.size = size;
    r.crypt = cyaes_relay_round16(size);
    r.conn = conn_id;
    r.done = done;
    r.user = user;
    return b->submit(std::move(r));
}

int cyaes_batcher_submit_open(cyaes_batcher* b, uint32_t slot, uint8_t* packet, uint32_t packet_bytes,
                              cyaes_done_fn done, void* user) {
    if (!b || !packet || packet_bytes < CYAES_RELAY_PAYLOAD_OFFSET) return CYAES_EINVAL;
    const uint32_t psize = (uint32_t)((packet[0] << 8) | packet[1]);  // BE u16 (cye_packet.cpp:82-86)
    const uint32_t pid = (uint32_t)((packet[2] << 8) | packet[3]);
    if (pid != CYAES_RELAY_FORWARD || psize + CYAES_RELAY_HEADSIZE != packet_bytes || psize < 8 ||
        (psize - 8) % 16)
        return CYAES_EINVAL;
    Req r{};
    int st = session_key(b, slot, &r.key);
    if (st) return st;
    r.op = CYAES_OP_RELAY_OPEN;
    r.in = packet;
    r.out = packet;
    r.size = packet_bytes;
    r.crypt = psize - 8u;  // relay_server.cpp:329: packet_size - sizeof(RelayForwardMsg)
    r.done = done;
    r.user = user;
    return b->submit(std::move(r));
}

int cyaes_batcher_flush(cyaes_batcher* b) {
    if (!b) return CYAES_EINVAL;
    std::unique_lock<std::mutex> lk(b->mu);
    const uint64_t target = b->submitted;
    b->flushers++;
    b->cv_submit.notify_all();
    b->cv_flush.wait(lk, [&] { return b->completed >= target; });
    b->flushers--;
    const int err = b->first_error;
    b->first_error = CYAES_OK;
    return err;
}

int cyaes_batcher_stats(cyaes_batcher* b, uint64_t out[6]) {
    if (!b || !out) return CYAES_EINVAL;
    std::lock_guard<std::mutex> lk(b->mu);
    out[0] = b->completed;
    out[1] = b->batches;
    out[2] = b->bytes;
    out[3] = b->max_batch;
    out[4] = b->errors;
    out[5] = b->submitted - b->completed;
    return CYAES_OK;
}

}  // extern "C"
