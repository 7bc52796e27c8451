// tools/bench_batcher.cpp -- relay-shaped load on the batching adapter
// (include/cyaes_batch.h), host to host (PCIe-inclusive).
//
// T "looper" threads each keep W requests in flight on their own session and
// resubmit from the completion callback's slot as soon as one finishes, the
// way a relay pipe would seal every chunk it reads (relay_local.cpp:189-206)
// or open every packet it receives (relay_server.cpp:329).  Reports requests/s,
// payload GiB/s and submit->callback latency percentiles as one JSON line, and
// for comparison the synchronous drop-in path (cyaes_cbc_encrypt, one packet
// per call, as the reference calls Rijndael::encrypt).
//
// Packet memory: by default every looper's slots are carved from one host
// region registered as a zero-copy pool (cyaes_batcher_register_pool), so the
// GPU gathers and scatters the packets itself; --pool 0 uses plain heap
// buffers (the bounce path: host copies in and out).  --submit pooled sends
// pool offsets (cyaes_batcher_submit_pooled) instead of pointers.  OPEN
// re-opens each slot's packet in place every round (the work is the same
// whatever the payload bytes are; --reopen-copy 1 restores the sealed packet
// with a host memcpy first, load-generator work).  --dump FILE writes every
// slot's input and output after a verification round (tests/ checks them
// against the relay restatement).
//
// usage: bench_batcher [--op seal|open|enc|dec] [--size B] [--threads T]
//                      [--window W] [--seconds S] [--batch-mb M] [--delay-us D]
//                      [--workers K] [--inflight I] [--bulk 0|1] [--pool 0|1]
//                      [--submit ptr|pooled] [--reopen-copy 0|1] [--dump FILE]
//                      [--complete callback|poll]
// --complete poll: the batcher runs with CYAES_BATCHER_POLL and each looper
// drains its own completion queue (cyaes_batcher_poll) in its loop instead of
// receiving one callback per packet.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "cyaes.h"
#include "cyaes_batch.h"
#include "cyaes_relay.h"

using Clock = std::chrono::steady_clock;

struct Slot {
    uint8_t *in = nullptr, *out = nullptr;  // in the looper's memory (a registered pool by default)
    uint32_t in_n = 0, out_n = 0;
    uint64_t in_off = 0, out_off = 0;       // offsets in the pool
    Clock::time_point t0;
    struct Looper* owner = nullptr;
};

struct Looper {
    cyaes_batcher* b = nullptr;
    uint32_t session = 0;
    int op = CYAES_OP_RELAY_SEAL;
    uint32_t size = 1472;
    uint8_t* mem = nullptr;  // the slots' buffers
    uint32_t pool = ~0u;     // registered pool id (~0u: not registered)
    bool pooled_submit = false, reopen_copy = false, poll = false;
    std::vector<Slot> slots;
    std::mutex mu;
    std::vector<Slot*> ready;  // completed, to resubmit
    std::vector<double> lat_us;
    std::atomic<uint64_t> done{0};
    int err = 0;
};

static void on_done(void* user, int status) {
    Slot* s = static_cast<Slot*>(user);
    Looper* L = s->owner;
    const double us = std::chrono::duration<double, std::micro>(Clock::now() - s->t0).count();
    std::lock_guard<std::mutex> lk(L->mu);
    if (status) L->err = status;
    if (L->lat_us.size() < 2000000) L->lat_us.push_back(us);
    L->ready.push_back(s);
    L->done.fetch_add(1, std::memory_order_relaxed);
}

static int submit(Looper* L, Slot* s) {
    s->t0 = Clock::now();
    switch (L->op) {
        case CYAES_OP_RELAY_SEAL:
            return cyaes_batcher_submit_seal(L->b, L->session, 7, s->in, L->size, s->out, on_done, s);
        case CYAES_OP_RELAY_OPEN:  // re-open the slot's packet in place: the work is the same every time
            if (L->reopen_copy) memcpy(s->out, s->in, s->in_n);
            return cyaes_batcher_submit_open(L->b, L->session, s->out, s->out_n, on_done, s);
        default:
            return cyaes_batcher_submit(L->b, L->op, L->session, s->in, s->out, L->size, on_done, s);
    }
}

static cyaes_batch_req make_req(Looper* L, Slot* s) {
    s->t0 = Clock::now();
    cyaes_done_fn cb = L->poll ? nullptr : on_done;
    switch (L->op) {
        case CYAES_OP_RELAY_SEAL:
            return {CYAES_OP_RELAY_SEAL, L->session, 7, s->in, s->out, L->size, cb, s};
        case CYAES_OP_RELAY_OPEN:
            if (L->reopen_copy) memcpy(s->out, s->in, s->in_n);
            return {CYAES_OP_RELAY_OPEN, L->session, 0, nullptr, s->out, s->out_n, cb, s};
        default:
            return {L->op, L->session, 0, s->in, s->out, L->size, cb, s};
    }
}

static cyaes_pool_req make_pool_req(Looper* L, Slot* s) {
    s->t0 = Clock::now();
    cyaes_done_fn cb = L->poll ? nullptr : on_done;
    switch (L->op) {
        case CYAES_OP_RELAY_SEAL:
            return {CYAES_OP_RELAY_SEAL, L->session, 7, L->pool, s->in_off, s->out_off, L->size, cb, s};
        case CYAES_OP_RELAY_OPEN:
            if (L->reopen_copy) memcpy(s->out, s->in, s->in_n);
            return {CYAES_OP_RELAY_OPEN, L->session, 0, L->pool, s->out_off, 0, s->out_n, cb, s};
        default:
            return {L->op, L->session, 0, L->pool, s->in_off, s->out_off, L->size, cb, s};
    }
}

static double pct(std::vector<double>& v, double p) {
    if (v.empty()) return 0;
    size_t k = std::min(v.size() - 1, (size_t)(p * (v.size() - 1)));
    std::nth_element(v.begin(), v.begin() + k, v.end());
    return v[k];
}

int main(int argc, char** argv) {
    std::string op = "seal";
    uint32_t size = 1472, threads = 8, window = 512, batch_mb = 32, delay_us = 100, workers = 4, inflight = 3, bulk = 1;
    uint32_t use_pool = 1, reopen_copy = 0;
    std::string submit_kind = "ptr", dump, complete = "callback";
    double seconds = 5;
    for (int i = 1; i + 1 < argc; i += 2) {
        std::string a = argv[i];
        if (a == "--op") op = argv[i + 1];
        else if (a == "--size") size = atoi(argv[i + 1]);
        else if (a == "--threads") threads = atoi(argv[i + 1]);
        else if (a == "--window") window = atoi(argv[i + 1]);
        else if (a == "--seconds") seconds = atof(argv[i + 1]);
        else if (a == "--batch-mb") batch_mb = atoi(argv[i + 1]);
        else if (a == "--delay-us") delay_us = atoi(argv[i + 1]);
        else if (a == "--workers") workers = atoi(argv[i + 1]);
        else if (a == "--inflight") inflight = atoi(argv[i + 1]);
        else if (a == "--bulk") bulk = atoi(argv[i + 1]);
        else if (a == "--pool") use_pool = atoi(argv[i + 1]);
        else if (a == "--submit") submit_kind = argv[i + 1];
        else if (a == "--reopen-copy") reopen_copy = atoi(argv[i + 1]);
        else if (a == "--dump") dump = argv[i + 1];
        else if (a == "--complete") complete = argv[i + 1];
    }
    const bool poll = complete == "poll";
    const bool pooled_submit = submit_kind == "pooled";
    if (pooled_submit && !use_pool) {
        fprintf(stderr, "--submit pooled needs --pool 1\n");
        return 1;
    }
    const int opc = op == "seal" ? CYAES_OP_RELAY_SEAL : op == "open" ? CYAES_OP_RELAY_OPEN
                    : op == "dec" ? CYAES_OP_DECRYPT : CYAES_OP_ENCRYPT;
    if ((opc == CYAES_OP_ENCRYPT || opc == CYAES_OP_DECRYPT) && size % 16) size = cyaes_relay_round16(size);
    if (opc >= CYAES_OP_RELAY_SEAL && size > CYAES_RELAY_MAX_CHUNK) size = CYAES_RELAY_MAX_CHUNK;

    cyaes_batcher_config cfg = {0, batch_mb << 20, delay_us, inflight, workers, 0, poll ? CYAES_BATCHER_POLL : 0u};
    cyaes_batcher* b = nullptr;
    int st = cyaes_batcher_create(&cfg, &b);
    if (st) {
        fprintf(stderr, "cyaes_batcher_create: %s\n", cyaes_strerror(st));
        return 1;
    }
    std::vector<Looper> loopers(threads);
    const uint32_t pkt = cyaes_relay_packet_bytes(size);
    const uint32_t in_n = opc == CYAES_OP_RELAY_OPEN ? pkt : size;
    const uint32_t out_n = opc >= CYAES_OP_RELAY_SEAL ? pkt : size;
    const uint64_t in_stride = (in_n + 63) & ~63u, out_stride = (out_n + 63) & ~63u;
    for (uint32_t t = 0; t < threads; t++) {
        Looper& L = loopers[t];
        L.b = b;
        L.op = opc;
        L.size = size;
        L.pooled_submit = pooled_submit;
        L.reopen_copy = reopen_copy != 0;
        L.poll = false;  // the warm-up and --dump rounds use callbacks (the loopers switch below)
        uint8_t key[16];
        for (int i = 0; i < 16; i++) key[i] = (uint8_t)(t * 16 + i);
        cyaes_batcher_session_open(b, key, &L.session);
        const uint64_t bytes = (uint64_t)window * (in_stride + out_stride);
        L.mem = static_cast<uint8_t*>(aligned_alloc(4096, (bytes + 4095) & ~4095ull));
        memset(L.mem, 0, bytes);
        if (use_pool && (st = cyaes_batcher_register_pool(b, L.mem, bytes, &L.pool)) != CYAES_OK) {
            fprintf(stderr, "cyaes_batcher_register_pool: %s\n", cyaes_strerror(st));
            return 1;
        }
        L.slots.resize(window);
        for (uint32_t w = 0; w < window; w++) {
            Slot& s = L.slots[w];
            s.owner = &L;
            s.in_off = (uint64_t)w * in_stride;
            s.out_off = (uint64_t)window * in_stride + (uint64_t)w * out_stride;
            s.in = L.mem + s.in_off;
            s.out = L.mem + s.out_off;
            s.in_n = in_n;
            s.out_n = out_n;
            for (size_t i = 0; i < in_n; i++) s.in[i] = (uint8_t)(i * 131 + w + 7 * t);
            if (opc == CYAES_OP_RELAY_OPEN) {
                cyaes_relay_build_forward(s.in, 7, s.in + 12, size);
                memcpy(s.out, s.in, in_n);
            }
        }
    }
    // Verification round (--dump): every slot once, then inputs and outputs to FILE.
    if (!dump.empty()) {
        for (auto& L : loopers)
            for (auto& s : L.slots) submit(&L, &s);
        cyaes_batcher_flush(b);
        FILE* f = fopen(dump.c_str(), "wb");
        if (!f) return 1;
        const uint32_t hdr[4] = {(uint32_t)opc, size, in_n, out_n};
        fwrite(hdr, sizeof(hdr), 1, f);
        for (auto& L : loopers) {
            uint8_t key[16];
            for (int i = 0; i < 16; i++) key[i] = (uint8_t)((&L - loopers.data()) * 16 + i);
            const uint32_t nslots = (uint32_t)L.slots.size();
            fwrite(key, 16, 1, f);
            fwrite(&nslots, 4, 1, f);
            for (auto& s : L.slots) {
                fwrite(s.in, 1, in_n, f);
                fwrite(s.out, 1, out_n, f);
            }
        }
        fclose(f);
        if (opc == CYAES_OP_RELAY_OPEN)  // restore the sealed packets for the timed rounds
            for (auto& L : loopers)
                for (auto& s : L.slots) memcpy(s.out, s.in, in_n);
    }
    // Warm-up: one window per looper.
    for (auto& L : loopers)
        for (auto& s : L.slots) submit(&L, &s);
    cyaes_batcher_flush(b);
    for (auto& L : loopers) {
        L.ready.clear();
        L.lat_us.clear();
        L.done = 0;
    }
    uint64_t st0[6];
    cyaes_batcher_stats(b, st0);

    std::atomic<bool> stop{false};
    const auto t0 = Clock::now();
    std::vector<std::thread> th;
    for (auto& L : loopers) {
        L.poll = poll;
        th.emplace_back([&L, &stop, bulk] {
            for (auto& s : L.slots) {
                if (L.poll) {  // (this thread's first submits: its completions come to its own queue)
                    cyaes_batch_req q = make_req(&L, &s);
                    cyaes_batcher_submit_many(L.b, &q, 1, nullptr);
                } else {
                    submit(&L, &s);
                }
            }
            std::vector<Slot*> again;
            std::vector<cyaes_batch_req> reqs;
            std::vector<cyaes_pool_req> preqs;
            std::vector<void*> users(L.slots.size());
            std::vector<int> sts(L.slots.size());
            while (!stop.load(std::memory_order_relaxed)) {
                if (L.poll) {  // drain this thread's completion queue
                    const uint32_t n = cyaes_batcher_poll(L.b, users.data(), sts.data(), (uint32_t)users.size());
                    const auto now = Clock::now();
                    for (uint32_t i = 0; i < n; i++) {
                        Slot* s = static_cast<Slot*>(users[i]);
                        if (sts[i]) L.err = sts[i];
                        if (L.lat_us.size() < 2000000)
                            L.lat_us.push_back(std::chrono::duration<double, std::micro>(now - s->t0).count());
                        again.push_back(s);
                    }
                    L.done.fetch_add(n, std::memory_order_relaxed);
                } else {
                    std::lock_guard<std::mutex> lk(L.mu);
                    again.swap(L.ready);
                }
                if (again.empty()) {
                    std::this_thread::sleep_for(std::chrono::microseconds(20));
                    continue;
                }
                if (bulk && L.pooled_submit) {  // one cyaes_batcher_submit_pooled per poll, by pool offsets
                    preqs.clear();
                    for (Slot* s : again) preqs.push_back(make_pool_req(&L, s));
                    cyaes_batcher_submit_pooled(L.b, preqs.data(), (uint32_t)preqs.size(), nullptr);
                } else if (bulk || L.poll) {  // one cyaes_batcher_submit_many per poll, as a relay looper would
                    reqs.clear();
                    for (Slot* s : again) reqs.push_back(make_req(&L, s));
                    cyaes_batcher_submit_many(L.b, reqs.data(), (uint32_t)reqs.size(), nullptr);
                } else {
                    for (Slot* s : again) submit(&L, s);
                }
                again.clear();
            }
        });
    }
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    stop = true;
    for (auto& t : th) t.join();
    const uint64_t counted = [&] {
        uint64_t n = 0;
        for (auto& L : loopers) n += L.done.load();
        return n;
    }();
    const double el = std::chrono::duration<double>(Clock::now() - t0).count();
    cyaes_batcher_flush(b);
    uint64_t st1[6];
    cyaes_batcher_stats(b, st1);
    std::vector<double> lat;
    int err = 0;
    for (auto& L : loopers) {
        lat.insert(lat.end(), L.lat_us.begin(), L.lat_us.end());
        err |= L.err;
    }
    const double payload = (double)(opc >= CYAES_OP_RELAY_SEAL ? cyaes_relay_round16(size) : size);
    const double batches = (double)(st1[1] - st0[1]);
    const double p50 = pct(lat, 0.5), p99 = pct(lat, 0.99);
    cyaes_batcher_destroy(b);
    for (auto& L : loopers) free(L.mem);

    // Synchronous drop-in for comparison: one packet per call (relay_local.cpp:206 shape).
    cyaes_key k;
    uint8_t key[16] = {0};
    cyaes_key_expand(key, &k);
    std::vector<uint8_t> buf(cyaes_relay_round16(size));
    cyaes_cbc_encrypt(&k, buf.data(), buf.data(), buf.size(), nullptr);
    int calls = 0;
    const auto s0 = Clock::now();
    while (std::chrono::duration<double>(Clock::now() - s0).count() < 1.0) {
        cyaes_cbc_encrypt(&k, buf.data(), buf.data(), buf.size(), nullptr);
        calls++;
    }
    const double sync_s = std::chrono::duration<double>(Clock::now() - s0).count();

    printf("{\"metric\": \"batcher %s requests/s host-to-host\", \"op\": \"%s\", \"size\": %u, \"threads\": %u, "
           "\"window\": %u, \"batch_mb\": %u, \"delay_us\": %u, \"workers\": %u, \"inflight\": %u, \"bulk\": %u, "
           "\"pool\": %u, \"submit\": \"%s\", \"complete\": \"%s\", \"seconds\": %.2f, \"requests\": %llu, "
           "\"requests_per_s\": %.0f, \"payload_gibs\": %.3f, \"mean_batch\": %.1f, \"lat_p50_us\": %.0f, "
           "\"lat_p99_us\": %.0f, \"errors\": %d, \"sync_dropin_calls_per_s\": %.0f, "
           "\"sync_dropin_gibs\": %.4f}\n",
           op.c_str(), op.c_str(), size, threads, window, batch_mb, delay_us, workers, inflight, bulk, use_pool,
           submit_kind.c_str(), complete.c_str(), el, (unsigned long long)counted,
           counted / el, counted * payload / el / (1u << 30), batches > 0 ? (st1[0] - st0[0]) / batches : 0.0, p50,
           p99, err, calls / sync_s, calls * (double)buf.size() / sync_s / (1u << 30));
    return err ? 2 : 0;
}
