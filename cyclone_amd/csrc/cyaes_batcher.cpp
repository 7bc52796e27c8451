// cyaes_batcher.cpp -- asynchronous batching adapter (include/cyaes_batch.h).
//
// Reference call pattern being replaced: synchronous per-packet
// Rijndael::encrypt / decrypt on the looper threads of samples/relay
// (relay_local.cpp:188-217, 365; relay_server.cpp:329, 453-481), with one
// Rijndael pair per pipe created after the DH handshake
// (relay_server.cpp:218-240) and deleted on close (:370-375).
//
// Threads: callers submit into one of kShards queues (the shard of the
// calling thread, so a thread's requests stay in order; one short shard lock
// per submit call, never the batcher's lock, and submit_many takes it once
// for many requests); the builder thread closes a batch when it is full, when
// its oldest request has waited max_delay_us, or when someone flushes -- it
// swaps the shard queues out and forms the batch outside every lock -- gathers it into a
// pinned staging buffer and launches H2D -> ragged encrypt -> ragged decrypt
// -> D2H on that stage's stream; the completion thread waits for the stage,
// scatters outputs, runs callbacks and recycles the stage.  Gather and
// scatter of large batches are split over `workers` threads (Pool).
// Staging layout of one batch (one H2D, one D2H):
//   [data: each request 16-B aligned][enc meta][dec meta][key schedules]
// A SEAL/OPEN request keeps its packet at data offset o + 4 so the payload
// (packet offset 12) sits at o + 16.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <functional>
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
    uint64_t seq;       // 1-based position in its shard's queue (flush watermark)
    uint8_t shard;
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

// Fixed worker threads for the gather / scatter copies of one stage: run(n, fn)
// calls fn(begin, end) over [0, n) in chunks, on the workers and the caller,
// and returns when all chunks are done.  One job at a time per pool.
class Pool {
  public:
    explicit Pool(int workers) {
        for (int i = 0; i < workers; i++) th_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    template <typename F>
    void run(size_t n, size_t chunk, F&& f) {
        if (th_.empty() || n <= chunk) {
            f(0, n);
            return;
        }
        std::function<void(size_t, size_t)> fn(std::forward<F>(f));
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &fn;
            n_ = n;
            chunk_ = chunk;
            next_.store(0);
            active_ = (int)th_.size();
            gen_++;
        }
        cv_.notify_all();
        work(fn, n, chunk);
        std::unique_lock<std::mutex> lk(mu_);
        cv_done_.wait(lk, [&] { return active_ == 0; });
        fn_ = nullptr;
    }

  private:
    void work(const std::function<void(size_t, size_t)>& fn, size_t n, size_t chunk) {
        for (;;) {
            const size_t b = next_.fetch_add(chunk);
            if (b >= n) return;
            fn(b, std::min(n, b + chunk));
        }
    }
    void loop() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            const auto* fn = fn_;
            const size_t n = n_, chunk = chunk_;
            lk.unlock();
            work(*fn, n, chunk);
            lk.lock();
            if (--active_ == 0) cv_done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, cv_done_;
    const std::function<void(size_t, size_t)>* fn_ = nullptr;
    size_t n_ = 0, chunk_ = 0;
    std::atomic<size_t> next_{0};
    int active_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// Requests per gather/scatter chunk: splitting pays only for large batches.
constexpr size_t kCopyChunk = 64;

// Submission shards: with one queue and one lock, 8 relay-style threads
// resubmitting ~1 M requests/s convoyed on the lock (tools/bench_batcher.cpp).
constexpr int kShards = 16;
struct alignas(64) Shard {
    std::mutex mu;
    std::vector<Req> q;
    uint64_t bytes = 0;     // data bytes queued in q
    uint64_t enqueued = 0;  // requests ever enqueued here (flush target, stats)
};
int my_shard() {
    static std::atomic<int> next{0};
    thread_local int s = next.fetch_add(1) % kShards;
    return s;
}
// Per-thread snapshot of a batcher's session table, refreshed when the table's
// version changes (open/close), so a submit takes no shared lock.
std::atomic<uint64_t> g_batcher_ids{1};
struct SessionSnap {
    uint64_t batcher = 0, version = 0;
    std::vector<std::shared_ptr<const Sched>> s;
};
thread_local SessionSnap t_snap;

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

// Per-thread phase times (ns), written only by their own thread, printed by
// cyaes_batcher_destroy when CYAES_BATCHER_PROFILE is set (after the joins).
struct Phases {
    int64_t wait = 0, take = 0, form = 0, layout = 0, gather = 0, submit = 0;  // builder
    int64_t sync = 0, scatter = 0, callbacks = 0, batches = 0, reqs = 0;       // completer
};

}  // namespace

struct cyaes_batcher {
    cyaes_batcher_config cfg{};
    cyaes_gpu* ctx = nullptr;
    uint64_t stage_cap = 0;
    std::vector<Stage> stages;

    // Submission: shard queues + counters (lock-free for submitters except their shard).
    std::array<Shard, kShards> shards;
    std::atomic<int64_t> queued_reqs{0}, queued_bytes{0};  // transiently negative while a drain races an enqueue
    std::atomic<int64_t> oldest_ns{0};  // submit time of the oldest queued request (0: none recorded)
    std::atomic<int> flushers{0};
    std::atomic<bool> stop{false};

    // Builder / completion hand-off, stats, flush (guarded by mu).
    std::mutex mu;
    std::condition_variable cv_submit, cv_free, cv_inflight, cv_flush;
    std::vector<Stage*> free_stages;
    std::deque<Stage*> inflight;
    bool builder_done = false;
    uint64_t completed = 0;
    // Per-shard completion watermark: the highest seq completed.  A shard's
    // requests complete in enqueue order (the builder appends each shard's
    // queue to carry in order, cuts batches in carry order, and batches
    // complete in launch order), so flush waits for every shard's watermark to
    // reach that shard's count at the call -- a global count could be reached
    // by later requests of other shards while earlier ones are still queued.
    std::array<uint64_t, kShards> done_seq{};
    uint64_t batches = 0, bytes = 0, max_batch = 0, errors = 0;
    int first_error = CYAES_OK;

    std::mutex smu;  // session table
    std::vector<std::shared_ptr<const Sched>> sessions;  // nullptr = free slot
    std::atomic<uint64_t> sessions_version{1};
    const uint64_t id = g_batcher_ids.fetch_add(1);
    const SessionSnap& snapshot();
    uint64_t enqueued_total();

    std::unique_ptr<Pool> gather_pool, scatter_pool;
    std::thread builder, completer;
    Phases pb, pc;  // builder / completer phase times
    struct Lists {  // builder-private scratch of launch(), reused across batches
        std::vector<uint64_t> eo, doff, o2;
        std::vector<uint32_t> el, ek, dl, dk, l2, k2, at;
        std::unordered_map<const Sched*, uint32_t> kidx;
        std::vector<const Sched*> klist;
    } lists;

    // Cost of a request in a stage: data + meta (16 B) + a schedule if its key is new to the batch.
    static uint64_t cost(const Req& r) { return r.data_bytes() + 16; }

    void build_loop();
    void complete_loop();
    int launch(Stage* st);
    int make(const cyaes_batch_req& q, const SessionSnap& ss, Req* r);
    void enqueue(Req* rs, size_t n, uint64_t nbytes);
};

void cyaes_batcher::build_loop() {
    std::vector<Req> carry;  // builder-private: taken from the shards, not yet batched (older than the shards)
    size_t cpos = 0;
    std::array<std::vector<Req>, kShards> spare;  // swapped into the shards: their capacity is recycled
    std::unordered_map<const Sched*, int> seen;
    for (;;) {
        Stage* st = nullptr;
        const int64_t tw = now_ns();
        {
            std::unique_lock<std::mutex> lk(mu);
            if (cpos == carry.size()) {
                carry.clear();
                cpos = 0;
                cv_submit.wait(lk, [&] { return stop || queued_reqs.load() > 0; });
                if (queued_reqs.load() <= 0) break;  // stop requested and drained
                // Let the batch fill: until it is full, the oldest request is due, or a flush/stop.
                const int64_t t = oldest_ns.load();
                const auto due = Clock::time_point(std::chrono::nanoseconds(t ? t : now_ns())) +
                                 std::chrono::microseconds(cfg.max_delay_us);
                cv_submit.wait_until(lk, due, [&] {
                    return stop || flushers.load() > 0 || queued_bytes.load() >= (int64_t)cfg.max_batch_bytes;
                });
            }
            cv_free.wait(lk, [&] { return !free_stages.empty(); });
            st = free_stages.back();
            free_stages.pop_back();
        }
        const int64_t tt = now_ns();
        pb.wait += tt - tw;
        // Take every shard's queue: a swap with a spare (empty, with capacity)
        // under each shard lock, then one move per request into carry.
        oldest_ns.store(0);
        int64_t took = 0, took_bytes = 0;
        for (int i = 0; i < kShards; i++) {
            Shard& sh = shards[i];
            {
                std::lock_guard<std::mutex> lk(sh.mu);
                if (sh.q.empty()) continue;
                sh.q.swap(spare[i]);
                took_bytes += (int64_t)sh.bytes;
                sh.bytes = 0;
            }
            std::vector<Req>& q = spare[i];
            took += (int64_t)q.size();
            if (cpos == carry.size()) {
                carry.clear();
                cpos = 0;
            }
            if (carry.empty()) carry.swap(q);  // q now holds carry's old (empty) buffer
            else carry.insert(carry.end(), std::make_move_iterator(q.begin()), std::make_move_iterator(q.end()));
            q.clear();
        }
        queued_reqs.fetch_sub(took);
        queued_bytes.fetch_sub(took_bytes);
        const int64_t tf = now_ns();
        pb.take += tf - tt;
        // Cut the batch: [cpos, end) of carry, bounded by max_batch_bytes and the stage.
        st->reqs.clear();
        uint64_t used = 0, data = 0;
        seen.clear();
        const Sched* last = nullptr;
        size_t end = cpos;
        for (; end < carry.size(); end++) {
            const Req& r = carry[end];
            bool new_key = false;
            if (r.key.get() != last) {
                last = r.key.get();
                new_key = seen.emplace(last, 0).second;
            }
            const uint64_t db = r.data_bytes();
            const uint64_t c = db + 16 + (new_key ? sizeof(Sched) : 0);
            if (end > cpos && (data + db > cfg.max_batch_bytes || used + c + 64 > stage_cap)) break;
            used += c;
            data += db;
        }
        if (cpos == 0 && end == carry.size()) {
            st->reqs.swap(carry);  // the whole carry: no moves (carry takes the stage's old buffer)
            carry.clear();
            cpos = 0;
        } else {
            st->reqs.insert(st->reqs.end(), std::make_move_iterator(carry.begin() + cpos),
                            std::make_move_iterator(carry.begin() + end));
            cpos = end;
        }
        if (st->reqs.empty()) {  // raced: nothing taken (cannot happen with took > 0 or carry)
            std::lock_guard<std::mutex> lk(mu);
            free_stages.push_back(st);
            continue;
        }
        pb.form += now_ns() - tf;
        st->status = launch(st);
        std::lock_guard<std::mutex> lk(mu);
        inflight.push_back(st);
        cv_inflight.notify_one();
    }
    std::lock_guard<std::mutex> lk(mu);
    builder_done = true;
    cv_inflight.notify_all();
}

// Gathers st->reqs into the stage and launches the batch on its stream.
int cyaes_batcher::launch(Stage* st) {
    const int64_t t0 = now_ns();
    const size_t n = st->reqs.size();
    st->off.resize(n);
    // Data section + per-direction lists.
    std::vector<uint64_t>& eo = lists.eo;
    std::vector<uint64_t>& doff = lists.doff;
    std::vector<uint32_t>&el = lists.el, &ek = lists.ek, &dl = lists.dl, &dk = lists.dk;
    for (auto* v : {&eo, &doff}) v->clear(), v->reserve(n);
    for (auto* v : {&el, &ek, &dl, &dk}) v->clear(), v->reserve(n);
    std::unordered_map<const Sched*, uint32_t>& kidx = lists.kidx;
    std::vector<const Sched*>& klist = lists.klist;
    kidx.clear();
    klist.clear();
    const Sched* last = nullptr;
    uint32_t k = 0;
    uint64_t pos = 0;
    for (size_t i = 0; i < n; i++) {  // layout pass (the copies run below, in parallel)
        const Req& r = st->reqs[i];
        st->off[i] = pos;
        const uint64_t coff = r.op >= CYAES_OP_RELAY_SEAL ? pos + 16 : pos;  // where the kernel works
        pos += r.data_bytes();
        if (r.crypt == 0) continue;  // size 0: a no-op (cyr_rijndael.cpp:600 loop never runs)
        if (r.key.get() != last) {  // requests come in per-thread runs: hash only on a change
            last = r.key.get();
            auto it = kidx.find(last);
            if (it == kidx.end()) {
                k = (uint32_t)klist.size();
                kidx.emplace(last, k);
                klist.push_back(last);
            } else {
                k = it->second;
            }
        }
        const bool dec = r.op == CYAES_OP_DECRYPT || r.op == CYAES_OP_RELAY_OPEN;
        (dec ? doff : eo).push_back(coff);
        (dec ? dl : el).push_back(r.crypt);
        (dec ? dk : ek).push_back(k);
    }
    st->data_end = pos;
    const int64_t t1 = now_ns();
    pb.layout += t1 - t0;
    gather_pool->run(n, kCopyChunk, [st](size_t b, size_t e) {
        for (size_t i = b; i < e; i++) {
            const Req& r = st->reqs[i];
            uint8_t* dst = st->h + st->off[i];
            switch (r.op) {
                case CYAES_OP_ENCRYPT:
                case CYAES_OP_DECRYPT:
                    memcpy(dst, r.in, r.size);
                    break;
                case CYAES_OP_RELAY_SEAL:  // relay_local.cpp:189-201: packet build + 0xCE padding
                    cyaes_relay_build_forward(dst + 4, r.conn, r.in, r.size);
                    break;
                case CYAES_OP_RELAY_OPEN:
                    memcpy(dst + 4, r.in, r.size);
                    break;
            }
        }
    });
    const int64_t t2 = now_ns();
    pb.gather += t2 - t1;
    // Encrypt runs one chain per lane and waterfalls over the distinct keys of
    // a wave (cyaes_kernels.hip, k_encrypt), so order its list by key: a wave
    // then sees one key, two at a boundary, instead of one per looper thread.
    // (Decrypt runs one payload per wave: one key per wave already.)
    // (Only for the lane-per-chain kernel: below its threshold the ragged
    // encrypt runs four lanes per chain with per-chain keys, and order does
    // not matter.)
    if (klist.size() > 1 && !eo.empty() && !cyaes::ragged_encrypt_is_quad(ctx, eo.size())) {
        // Stable counting sort by key index (key indices are dense: 0..klist.size()-1).
        std::vector<uint64_t>& o2 = lists.o2;
        std::vector<uint32_t>&l2 = lists.l2, &k2 = lists.k2, &at = lists.at;
        o2.resize(eo.size());
        l2.resize(el.size());
        k2.resize(ek.size());
        at.assign(klist.size() + 1, 0);
        for (uint32_t x : ek) at[x + 1]++;
        for (size_t j = 1; j < at.size(); j++) at[j] += at[j - 1];
        for (size_t i = 0; i < ek.size(); i++) {
            const uint32_t d = at[ek[i]]++;
            o2[d] = eo[i], l2[d] = el[i], k2[d] = ek[i];
        }
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
    pb.submit += now_ns() - t2;
    return map_err(e);
}

// Copies request i's result out of the stage into the caller's buffer.
static void scatter(Stage* st, size_t i) {
    const Req& r = st->reqs[i];
    const uint8_t* src = st->h + st->off[i];
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

void cyaes_batcher::complete_loop() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
        cv_inflight.wait(lk, [&] { return !inflight.empty() || builder_done; });
        if (inflight.empty()) break;
        Stage* st = inflight.front();
        inflight.pop_front();
        lk.unlock();
        int status = st->status;
        const int64_t t0 = now_ns();
        if (status == CYAES_OK) status = map_err(hipEventSynchronize(st->done));
        // A stage whose submit failed part-way may still have copies or kernels in
        // flight on its buffers: drain its stream before the stage is reused.
        if (status != CYAES_OK) (void)hipStreamSynchronize(st->stream);
        const int64_t t1 = now_ns();
        pc.sync += t1 - t0;
        if (status == CYAES_OK)
            scatter_pool->run(st->reqs.size(), kCopyChunk, [st](size_t b, size_t e) {
                for (size_t i = b; i < e; i++) scatter(st, i);
            });
        const int64_t t2 = now_ns();
        pc.scatter += t2 - t1;
        // Callbacks on this thread, in batch order.  (A/B: spreading them over
        // the scatter workers by submission shard was slower under the
        // relay-shaped load of tools/bench_batcher.cpp: the callbacks then
        // contend with the submitting threads.)
        uint64_t nbytes = 0;
        std::array<uint64_t, kShards> hi{};
        for (const Req& r : st->reqs) {
            nbytes += r.crypt;
            hi[r.shard] = std::max(hi[r.shard], r.seq);
            if (r.done) r.done(r.user, status);
        }
        const size_t nreq = st->reqs.size();
        st->reqs.clear();  // drops the schedule references
        pc.callbacks += now_ns() - t2;
        pc.batches++;
        pc.reqs += (int64_t)nreq;
        lk.lock();
        completed += nreq;
        for (int i = 0; i < kShards; i++) done_seq[i] = std::max(done_seq[i], hi[i]);
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

// This thread's snapshot of the session table (refreshed under smu when an
// open/close has bumped the version since this thread last looked).
const SessionSnap& cyaes_batcher::snapshot() {
    SessionSnap& ss = t_snap;
    const uint64_t v = sessions_version.load(std::memory_order_acquire);
    if (ss.batcher != id || ss.version != v) {
        std::lock_guard<std::mutex> lk(smu);
        ss.s = sessions;
        ss.batcher = id;
        ss.version = sessions_version.load(std::memory_order_relaxed);
    }
    return ss;
}

uint64_t cyaes_batcher::enqueued_total() {
    uint64_t n = 0;
    for (Shard& sh : shards) {
        std::lock_guard<std::mutex> lk(sh.mu);
        n += sh.enqueued;
    }
    return n;
}

// Validates one request and pins its session's schedule.
int cyaes_batcher::make(const cyaes_batch_req& q, const SessionSnap& ss, Req* r) {
    *r = Req{};
    switch (q.op) {
        case CYAES_OP_ENCRYPT:
        case CYAES_OP_DECRYPT:
            if (q.size % 16 || q.size > cfg.max_batch_bytes || (q.size && (!q.in || !q.out))) return CYAES_EINVAL;
            r->size = r->crypt = q.size;
            r->in = q.in;
            r->out = q.out;
            break;
        case CYAES_OP_RELAY_SEAL:
            if (!q.out || q.size > CYAES_RELAY_MAX_CHUNK || (q.size && !q.in)) return CYAES_EINVAL;
            r->in = q.in;
            r->out = q.out;
            r->size = q.size;
            r->crypt = cyaes_relay_round16(q.size);
            r->conn = q.conn_id;
            break;
        case CYAES_OP_RELAY_OPEN: {
            uint8_t* packet = q.out ? q.out : const_cast<uint8_t*>(q.in);
            if (!packet || q.size < CYAES_RELAY_PAYLOAD_OFFSET) return CYAES_EINVAL;
            const uint32_t psize = (uint32_t)((packet[0] << 8) | packet[1]);  // BE u16 (cye_packet.cpp:82-86)
            const uint32_t pid = (uint32_t)((packet[2] << 8) | packet[3]);
            if (pid != CYAES_RELAY_FORWARD || psize + CYAES_RELAY_HEADSIZE != q.size || psize < 8 || (psize - 8) % 16)
                return CYAES_EINVAL;
            r->in = packet;
            r->out = packet;
            r->size = q.size;
            r->crypt = psize - 8u;  // relay_server.cpp:329: packet_size - sizeof(RelayForwardMsg)
            break;
        }
        default:
            return CYAES_EINVAL;
    }
    if (q.slot >= ss.s.size() || !ss.s[q.slot]) return CYAES_ERANGE;
    r->op = (uint8_t)q.op;
    r->key = ss.s[q.slot];
    r->done = q.done;
    r->user = q.user;
    return CYAES_OK;
}

// Appends n requests to the calling thread's shard (one lock) and wakes the
// builder when the queue was empty or the batch is now full.
void cyaes_batcher::enqueue(Req* rs, size_t n, uint64_t nbytes) {
    if (n == 0) return;
    const auto t = Clock::now();
    const int s = my_shard();
    Shard& sh = shards[s];
    {
        std::lock_guard<std::mutex> lk(sh.mu);
        for (size_t i = 0; i < n; i++) {
            rs[i].t = t;
            rs[i].seq = sh.enqueued + i + 1;
            rs[i].shard = (uint8_t)s;
            sh.q.push_back(std::move(rs[i]));
        }
        sh.bytes += nbytes;
        sh.enqueued += n;
    }
    if (oldest_ns.load(std::memory_order_relaxed) == 0) {  // a plain load while a time is recorded
        int64_t zero = 0;
        oldest_ns.compare_exchange_strong(zero, std::chrono::duration_cast<std::chrono::nanoseconds>(
                                                    t.time_since_epoch()).count());
    }
    const int64_t before = queued_reqs.fetch_add((int64_t)n);
    const int64_t b0 = queued_bytes.fetch_add((int64_t)nbytes), cap = cfg.max_batch_bytes;
    if (before <= 0 || (b0 < cap && b0 + (int64_t)nbytes >= cap)) {
        std::lock_guard<std::mutex> lk(mu);  // orders the wake-up after the builder's predicate check
        cv_submit.notify_one();
    }
}

extern "C" {

int cyaes_batcher_create(const cyaes_batcher_config* cfg, cyaes_batcher** out) {
    if (!cfg || !out) return CYAES_EINVAL;
    *out = nullptr;
    cyaes_batcher_config c = *cfg;
    if (c.max_batch_bytes == 0) c.max_batch_bytes = 32u << 20;
    if (c.max_delay_us == 0) c.max_delay_us = 100;
    if (c.inflight == 0) c.inflight = 3;
    if (c.workers == 0) c.workers = 4;
    if (c.max_batch_bytes < 4096 || c.max_batch_bytes > (1u << 30) || c.inflight > 16 || c.workers > 64)
        return CYAES_EINVAL;
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
    b->gather_pool.reset(new Pool((int)c.workers - 1));  // + the builder thread itself
    b->scatter_pool.reset(new Pool((int)c.workers - 1)); // + the completion thread itself
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
        b->stop.store(true);
    }
    b->cv_submit.notify_all();
    if (b->builder.joinable()) b->builder.join();
    if (b->completer.joinable()) b->completer.join();
    if (getenv("CYAES_BATCHER_PROFILE") && b->pc.batches) {
        const Phases &B = b->pb, &C = b->pc;
        const double nb = (double)C.batches, us = 1e-3;
        fprintf(stderr,
                "[cyaes_batcher] %lld batches, %.0f reqs/batch; per batch (us): builder wait %.0f take %.0f form %.0f "
                "layout %.0f gather %.0f submit %.0f | completer sync %.0f scatter %.0f callbacks %.0f\n",
                (long long)C.batches, C.reqs / nb, B.wait * us / nb, B.take * us / nb, B.form * us / nb,
                B.layout * us / nb, B.gather * us / nb, B.submit * us / nb, C.sync * us / nb, C.scatter * us / nb,
                C.callbacks * us / nb);
    }
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
    std::lock_guard<std::mutex> lk(b->smu);
    size_t i = 0;
    while (i < b->sessions.size() && b->sessions[i]) i++;
    if (i == b->sessions.size()) b->sessions.emplace_back();
    b->sessions[i] = std::move(s);
    b->sessions_version.fetch_add(1, std::memory_order_release);
    *slot = (uint32_t)i;
    return CYAES_OK;
}

int cyaes_batcher_session_close(cyaes_batcher* b, uint32_t slot) {
    if (!b) return CYAES_EINVAL;
    std::lock_guard<std::mutex> lk(b->smu);
    if (slot >= b->sessions.size() || !b->sessions[slot]) return CYAES_ERANGE;
    b->sessions[slot].reset();
    b->sessions_version.fetch_add(1, std::memory_order_release);
    return CYAES_OK;
}

static int submit_one(cyaes_batcher* b, const cyaes_batch_req& q) {
    if (b->stop.load()) return CYAES_EINVAL;
    Req r;
    const int st = b->make(q, b->snapshot(), &r);
    if (st) return st;
    b->enqueue(&r, 1, r.data_bytes());
    return CYAES_OK;
}

int cyaes_batcher_submit(cyaes_batcher* b, int op, uint32_t slot, const uint8_t* in, uint8_t* out, size_t size,
                         cyaes_done_fn done, void* user) {
    if (!b || (op != CYAES_OP_ENCRYPT && op != CYAES_OP_DECRYPT) || size > 0xFFFFFFFFu) return CYAES_EINVAL;
    return submit_one(b, cyaes_batch_req{op, slot, 0, in, out, (uint32_t)size, done, user});
}

int cyaes_batcher_submit_seal(cyaes_batcher* b, uint32_t slot, int32_t conn_id, const uint8_t* payload,
                              uint32_t size, uint8_t* packet_out, cyaes_done_fn done, void* user) {
    if (!b) return CYAES_EINVAL;
    return submit_one(b, cyaes_batch_req{CYAES_OP_RELAY_SEAL, slot, conn_id, payload, packet_out, size, done, user});
}

int cyaes_batcher_submit_open(cyaes_batcher* b, uint32_t slot, uint8_t* packet, uint32_t packet_bytes,
                              cyaes_done_fn done, void* user) {
    if (!b) return CYAES_EINVAL;
    return submit_one(b, cyaes_batch_req{CYAES_OP_RELAY_OPEN, slot, 0, packet, packet, packet_bytes, done, user});
}

int cyaes_batcher_submit_many(cyaes_batcher* b, const cyaes_batch_req* reqs, uint32_t n, int* status) {
    if (!b || (n && !reqs)) return CYAES_EINVAL;
    if (b->stop.load()) return CYAES_EINVAL;
    std::vector<Req> rs(n);
    size_t k = 0;
    uint64_t nbytes = 0;
    int first = CYAES_OK;
    const SessionSnap& ss = b->snapshot();
    for (uint32_t i = 0; i < n; i++) {
        const int st = b->make(reqs[i], ss, &rs[k]);
        if (status) status[i] = st;
        if (st) {
            if (first == CYAES_OK) first = st;
            continue;
        }
        nbytes += rs[k].data_bytes();
        k++;
    }
    b->enqueue(rs.data(), k, nbytes);
    return first;
}

int cyaes_batcher_flush(cyaes_batcher* b) {
    if (!b) return CYAES_EINVAL;
    std::array<uint64_t, kShards> target;  // every shard's queue length at the call
    for (int i = 0; i < kShards; i++) {
        std::lock_guard<std::mutex> sl(b->shards[i].mu);
        target[i] = b->shards[i].enqueued;
    }
    std::unique_lock<std::mutex> lk(b->mu);
    b->flushers.fetch_add(1);
    b->cv_submit.notify_all();
    b->cv_flush.wait(lk, [&] {
        for (int i = 0; i < kShards; i++)
            if (b->done_seq[i] < target[i]) return false;
        return true;
    });
    b->flushers.fetch_sub(1);
    const int err = b->first_error;
    b->first_error = CYAES_OK;
    return err;
}

int cyaes_batcher_stats(cyaes_batcher* b, uint64_t out[6]) {
    if (!b || !out) return CYAES_EINVAL;
    std::lock_guard<std::mutex> lk(b->mu);  // completed cannot grow while held: pending >= 0
    out[0] = b->completed;
    out[1] = b->batches;
    out[2] = b->bytes;
    out[3] = b->max_batch;
    out[4] = b->errors;
    out[5] = b->enqueued_total() - b->completed;
    return CYAES_OK;
}

}  // extern "C"
