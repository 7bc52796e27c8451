// cyaes_batcher.cpp -- asynchronous batching adapter (include/cyaes_batch.h).
//
// Reference call pattern being replaced: synchronous per-packet
// Rijndael::encrypt / decrypt on the looper threads of samples/relay
// (relay_local.cpp:188-217, 365; relay_server.cpp:329, 453-481), with one
// Rijndael pair per pipe created after the DH handshake
// (relay_server.cpp:218-240) and deleted on close (:370-375).
//
// Zero-copy design (round 3):
//  * Callers register their packet memory once as pools (hipHostRegister,
//    mapped).  A request is a 40-byte descriptor (BatchDesc) naming its input
//    and output by device address; the GPU gathers the inputs from the pools
//    into an HBM stage, builds SEAL packets there, runs the ragged AES kernels
//    and scatters the outputs back into the pools (cyaes_batch_kernels.hip).
//    The host copies no payload byte.  Requests outside every pool go through
//    the batcher's pinned bounce buffer (host copies in and out: the legacy
//    path, same results).
//  * Keys: a session slot maps to a row of a device key table written once at
//    open.  A closed row is reused only after every request enqueued before
//    the close has completed (per-shard completion watermarks), so requests
//    already submitted keep their key.
//  * Submitters append descriptors to their thread's shard (one short lock per
//    submit call); the builder swaps the shard queues out and lays the batch
//    out with a few stores per request (encrypt-type descriptors first, then
//    decrypt-type, so each direction is one ragged list).
//  * One in-order pipeline stream (streams sharing a hardware queue serialise
//    anyway): H2D of batch k+1's descriptors; one move kernel that scatters
//    batch k's outputs while it gathers batch k+1's inputs, so both PCIe
//    directions run at once; batch k's completion event; batch k+1's AES
//    kernels, alone on the GPU.  An idle builder flushes the last scatter.
//  * The completion thread waits for each batch's event and runs the
//    callbacks, one job per shard on the worker pool, each shard's callbacks
//    in its submission order.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "cyaes.h"
#include "cyaes_batch.h"
#include "cyaes_internal.h"
#include "cyaes_relay.h"
#include "cyaes_tables.h"

using cyaes::BatchDesc;

namespace {

using Clock = std::chrono::steady_clock;

uint64_t up16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

// A batch whose longest encrypt-type payload has at least this many bytes runs
// its two directions side by side (cyaes::ragged_duplex_batch).
constexpr uint32_t kDuplexMinChain = 16384;

int map_err(hipError_t e) {
    if (e == hipSuccess) return CYAES_OK;
    return (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? CYAES_ENOMEM : CYAES_EDEVICE;
}

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

constexpr int kShards = 16;            // submission shards (a thread's shard is fixed)
constexpr uint32_t kMaxReqs = 65536;   // requests per batch
constexpr int kMaxPools = 64;
constexpr uint32_t kNoRow = ~0u;
constexpr uint32_t kSchedBytes = cyaes::kSchedWords * 4;
constexpr size_t kCopyChunk = 64;      // bounce copies per worker job (one atomic per chunk, not per copy)

// Stage bytes of a request's data in HBM: relay packets keep their payload at
// stage + 16 (16-B aligned), with the packet's 12 header bytes before it.
uint64_t stage_bytes(const BatchDesc& d) { return up16(d.op >= cyaes::kOpRelaySeal ? 16 + d.crypt : d.size); }
// Bounce bytes of a request outside the pools: one region for input and output.
uint64_t bounce_bytes(const BatchDesc& d) {
    switch (d.op) {
        case cyaes::kOpRelaySeal: return up16(CYAES_RELAY_PAYLOAD_OFFSET + d.crypt);  // chunk in, packet out
        default: return up16(d.size);                                                 // data / packet
    }
}

struct Cb {
    cyaes_done_fn done;
    void* user;
};

// A queued request.  d.src / d.dst are device addresses for pooled requests;
// for a bounced one they are the caller's host pointers until the builder
// moves the request into a stage's bounce buffer.
struct Pend {
    BatchDesc d;
    Cb cb;
    bool bounce;
};

// Fixed worker threads: run(n, fn) calls fn(i) for i in [0, n) on the workers
// and the caller, and returns when all are done.  One job at a time.
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
    void run(size_t n, const std::function<void(size_t)>& fn) {
        if (th_.empty() || n <= 1) {
            for (size_t i = 0; i < n; i++) fn(i);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &fn;
            n_ = n;
            next_.store(0);
            active_ = (int)th_.size();
            gen_++;
        }
        cv_.notify_all();
        work(fn, n);
        std::unique_lock<std::mutex> lk(mu_);
        cv_done_.wait(lk, [&] { return active_ == 0; });
        fn_ = nullptr;
    }

  private:
    void work(const std::function<void(size_t)>& fn, size_t n) {
        for (;;) {
            const size_t i = next_.fetch_add(1);
            if (i >= n) return;
            fn(i);
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
            const size_t n = n_;
            lk.unlock();
            work(*fn, n);
            lk.lock();
            if (--active_ == 0) cv_done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, cv_done_;
    const std::function<void(size_t)>* fn_ = nullptr;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    int active_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

struct Done {
    void* user;
    int status;
};
struct alignas(64) Shard {
    std::mutex mu;
    std::vector<Pend> q;
    uint64_t bytes = 0;     // stage bytes queued in q
    uint64_t enqueued = 0;  // requests ever enqueued here (flush targets, key-row stamps, stats)
    alignas(64) std::mutex cmu;  // CYAES_BATCHER_POLL completion queue
    std::deque<Done> cq;
};
int my_shard() {
    static std::atomic<int> next{0};
    thread_local int s = next.fetch_add(1) % kShards;
    return s;
}

struct PoolEnt {
    uint8_t* host = nullptr;
    uint64_t dev = 0;
    uint64_t bytes = 0;
    bool live = false;
};

// Per-thread snapshot of a batcher's session rows and pools, refreshed when
// either table's version changes, so a submit takes no shared lock.
std::atomic<uint64_t> g_batcher_ids{1};
struct Snap {
    uint64_t batcher = 0, sver = 0, pver = 0;
    std::vector<uint32_t> rows;  // slot -> key row (kNoRow: closed)
    struct Range {
        uintptr_t lo, hi;
        uint64_t dev;
    };
    std::vector<Range> pools;    // live pools by host address
    std::vector<PoolEnt> by_id;  // pool id -> entry (cyaes_batcher_submit_pooled)
};
thread_local Snap t_snap;

struct Seg {  // a shard's run of callbacks inside one batch
    uint8_t shard;
    uint32_t begin, end;  // into Stage::cbs
    uint64_t last_seq;    // that shard's sequence number of its last request here
};
struct BounceOut {  // completer copy of a bounced request's output
    uint8_t* to;
    const uint8_t* from;
    uint32_t bytes;
};

struct Stage {
    BatchDesc* h_enc = nullptr;  // pinned: encrypt-type descriptors [0, kMaxReqs)
    BatchDesc* h_dec = nullptr;  // pinned: decrypt-type descriptors [0, kMaxReqs)
    uint8_t* h_bounce = nullptr; // pinned, mapped
    uint64_t bounce_dev = 0;
    uint8_t* d_mem = nullptr;    // device: descriptors | lists | data
    BatchDesc* d_desc = nullptr;
    uint64_t* d_offs = nullptr;
    uint32_t *d_nb = nullptr, *d_kid = nullptr;
    uint8_t* d_data = nullptr;
    hipEvent_t done = nullptr;  // recorded after the batch's scatter
    uint32_t ne = 0, nd = 0;
    uint32_t emax = 0;   // the longest encrypt-type payload (bytes)
    uint64_t dbytes = 0; // decrypt-type payload bytes
    uint64_t bytes = 0;  // payload bytes en/decrypted (stats)
    std::vector<Cb> cbs;
    std::vector<Seg> segs;
    std::vector<BounceOut> bouts;
    int status = CYAES_OK;
};

struct Phases {  // per-batch phase times (ns), CYAES_BATCHER_PROFILE
    int64_t wait = 0, take = 0, layout = 0, copy_in = 0, submit = 0;
    int64_t sync = 0, copy_out = 0, callbacks = 0, batches = 0, reqs = 0;
};

}  // namespace

struct cyaes_batcher {
    cyaes_batcher_config cfg{};
    cyaes_gpu* ctx = nullptr;
    uint64_t data_cap = 0, bounce_cap = 0;
    int move_waves = 0;
    std::vector<Stage> stages;
    hipStream_t pipe = nullptr;  // the device pipeline (builder thread only)
    Stage* pending = nullptr;    // launched, its scatter not yet (builder thread only)

    std::array<Shard, kShards> shards;
    std::atomic<int64_t> queued_reqs{0}, queued_bytes{0};
    std::atomic<int64_t> oldest_ns{0};
    std::atomic<int> flushers{0};
    std::atomic<bool> stop{false};

    std::mutex mu;  // builder / completer hand-off, stats, flush
    std::condition_variable cv_submit, cv_free, cv_inflight, cv_flush;
    std::vector<Stage*> free_stages;
    std::deque<Stage*> inflight;
    std::vector<Cb> run_cbs;    // completer: the callbacks of the batch being completed
    std::vector<Seg> run_segs;
    bool builder_done = false;
    uint64_t completed = 0, batches = 0, bytes = 0, max_batch = 0, errors = 0;
    int first_error = CYAES_OK;
    std::array<uint64_t, kShards> done_seq{};  // per shard: requests completed (they complete in order)

    // Sessions: slot -> device key-table row.
    std::mutex smu;
    uint32_t key_cap = 0;
    uint32_t* d_keys = nullptr;
    std::vector<uint32_t> slot_row;
    std::vector<uint32_t> free_rows;
    uint32_t next_row = 0;
    struct Retired {
        uint32_t row;
        std::array<uint64_t, kShards> stamp;  // shard enqueue counts at the close
    };
    std::vector<Retired> retired;
    std::atomic<uint64_t> sessions_version{1};

    // Pools.
    std::mutex pmu;
    std::array<PoolEnt, kMaxPools> pools{};
    // pool id -> the registrations holding its pages (cyaes_pins.cpp: shared
    // with other pools, of this batcher or another, that sit on the same pages)
    std::array<cyaes::PinHold, kMaxPools> pool_pins;
    std::atomic<uint64_t> pools_version{1};

    const uint64_t id = g_batcher_ids.fetch_add(1);
    // One job at a time per pool: the builder's (bounce input copies) and the
    // completion side's (bounce output copies, callbacks) run concurrently.
    std::unique_ptr<Pool> in_pool, workers;
    std::thread builder, completer;
    Phases pb, pc;

    const Snap& snapshot();
    int make(const cyaes_batch_req& q, const Snap& ss, Pend* p);
    int make_pooled(const cyaes_pool_req& q, const Snap& ss, Pend* p);
    template <typename MakeAll>
    int enqueue(MakeAll&& make_all);
    void build_loop();
    void complete_loop();
    int launch(Stage* st);
    void flush_pending();
    void hand_off(Stage* st);
    int wait_enqueued(const std::array<uint64_t, kShards>& target);
    void wait_done(const std::array<uint64_t, kShards>& target);
};

// ---- submission --------------------------------------------------------------
const Snap& cyaes_batcher::snapshot() {
    Snap& ss = t_snap;
    const uint64_t sv = sessions_version.load(std::memory_order_acquire);
    const uint64_t pv = pools_version.load(std::memory_order_acquire);
    if (ss.batcher != id || ss.sver != sv) {
        std::lock_guard<std::mutex> lk(smu);
        ss.rows = slot_row;
        ss.sver = sessions_version.load(std::memory_order_relaxed);
    }
    if (ss.batcher != id || ss.pver != pv) {
        std::lock_guard<std::mutex> lk(pmu);
        ss.pools.clear();
        ss.by_id.assign(pools.begin(), pools.end());
        for (const PoolEnt& e : pools)
            if (e.live) ss.pools.push_back({(uintptr_t)e.host, (uintptr_t)e.host + e.bytes, e.dev});
        std::sort(ss.pools.begin(), ss.pools.end(), [](const Snap::Range& a, const Snap::Range& b) { return a.lo < b.lo; });
        ss.pver = pools_version.load(std::memory_order_relaxed);
    }
    ss.batcher = id;
    return ss;
}

// Device address of host range [p, p + n) if a registered pool holds all of it, else 0.
static uint64_t pool_dev(const Snap& ss, const void* p, uint64_t n) {
    const uintptr_t a = (uintptr_t)p;
    auto it = std::upper_bound(ss.pools.begin(), ss.pools.end(), a,
                               [](uintptr_t x, const Snap::Range& r) { return x < r.lo; });
    if (it == ss.pools.begin()) return 0;
    --it;
    if (a < it->lo || a + n > it->hi || a + n < a) return 0;
    return it->dev + (a - it->lo);
}

// Validates one pointer request; finds its pools (or marks it bounced).
int cyaes_batcher::make(const cyaes_batch_req& q, const Snap& ss, Pend* p) {
    *p = Pend{};
    BatchDesc& d = p->d;
    const uint8_t *in = nullptr, *out = nullptr;
    uint64_t in_n = 0, out_n = 0;
    switch (q.op) {
        case CYAES_OP_ENCRYPT:
        case CYAES_OP_DECRYPT:
            if (q.size % 16 || q.size > cfg.max_batch_bytes || (q.size && (!q.in || !q.out))) return CYAES_EINVAL;
            d.size = d.crypt = q.size;
            in = q.in, out = q.out, in_n = out_n = q.size;
            break;
        case CYAES_OP_RELAY_SEAL:
            if (!q.out || q.size > CYAES_RELAY_MAX_CHUNK || (q.size && !q.in)) return CYAES_EINVAL;
            d.size = q.size;
            d.crypt = cyaes_relay_round16(q.size);
            d.conn = q.conn_id;
            in = q.in, out = q.out, in_n = q.size, out_n = CYAES_RELAY_PAYLOAD_OFFSET + d.crypt;
            break;
        case CYAES_OP_RELAY_OPEN: {
            uint8_t* packet = q.out ? q.out : const_cast<uint8_t*>(q.in);
            if (!packet || q.size < CYAES_RELAY_PAYLOAD_OFFSET) return CYAES_EINVAL;
            const uint32_t psize = (uint32_t)((packet[0] << 8) | packet[1]);  // BE u16 (cye_packet.cpp:82-86)
            const uint32_t pid = (uint32_t)((packet[2] << 8) | packet[3]);
            if (pid != CYAES_RELAY_FORWARD || psize + CYAES_RELAY_HEADSIZE != q.size || psize < 8 || (psize - 8) % 16)
                return CYAES_EINVAL;
            d.size = q.size;
            d.crypt = psize - 8u;  // relay_server.cpp:329: packet_size - sizeof(RelayForwardMsg)
            in = out = packet, in_n = out_n = q.size;
            break;
        }
        default:
            return CYAES_EINVAL;
    }
    if (q.slot >= ss.rows.size() || ss.rows[q.slot] == kNoRow) return CYAES_ERANGE;
    d.op = (uint32_t)q.op;
    d.key = ss.rows[q.slot];
    p->cb = Cb{q.done, q.user};
    const uint64_t ds = in_n ? pool_dev(ss, in, in_n) : 1, dd = out_n ? pool_dev(ss, out, out_n) : 1;
    if (ds && dd) {  // zero-copy: the GPU reads and writes the caller's pool memory itself
        d.src = in_n ? ds : 0;
        d.dst = out_n ? dd : 0;
    } else {
        p->bounce = true;
        d.src = (uint64_t)(uintptr_t)in;
        d.dst = (uint64_t)(uintptr_t)out;
    }
    return CYAES_OK;
}

int cyaes_batcher::make_pooled(const cyaes_pool_req& q, const Snap& ss, Pend* p) {
    if (q.pool >= ss.by_id.size() || !ss.by_id[q.pool].live) return CYAES_EINVAL;
    const PoolEnt& e = ss.by_id[q.pool];
    if (q.in_off > e.bytes || (q.op != CYAES_OP_RELAY_OPEN && q.out_off > e.bytes)) return CYAES_EINVAL;
    // OPEN reads the packet header in make(): the whole packet must lie in the pool first
    if (q.op == CYAES_OP_RELAY_OPEN && (q.size < CYAES_RELAY_PAYLOAD_OFFSET || q.size > e.bytes - q.in_off))
        return CYAES_EINVAL;
    cyaes_batch_req r{q.op, q.slot, q.conn_id, e.host + q.in_off,
                      q.op == CYAES_OP_RELAY_OPEN ? e.host + q.in_off : e.host + q.out_off, q.size, q.done, q.user};
    const int st = make(r, ss, p);
    if (st == CYAES_OK && p->bounce) return CYAES_EINVAL;  // the request runs past its pool's end
    return st;
}

// Builds this thread's requests against its snapshot and appends them to its
// shard under one lock.  The snapshot is re-checked under the shard lock: a
// close stamps its key row with the shard counts (taking each shard lock), so
// a request either enqueued before that stamp (and keeps the row alive) or
// sees the new version and is rebuilt against it (ERANGE for a closed slot).
template <typename MakeAll>
int cyaes_batcher::enqueue(MakeAll&& make_all) {
    thread_local std::vector<Pend> ps;
    const int s = my_shard();
    Shard& sh = shards[s];
    for (;;) {
        const Snap& ss = snapshot();
        ps.clear();
        uint64_t nbytes = 0;
        const int first = make_all(ss, ps, nbytes);
        if (ps.empty()) return first;
        int64_t before, b0;
        {
            std::lock_guard<std::mutex> lk(sh.mu);
            if (sessions_version.load(std::memory_order_acquire) != ss.sver ||
                pools_version.load(std::memory_order_acquire) != ss.pver)
                continue;  // a session or pool changed since the snapshot: rebuild
            sh.q.insert(sh.q.end(), ps.begin(), ps.end());
            sh.bytes += nbytes;
            sh.enqueued += ps.size();
        }
        if (oldest_ns.load(std::memory_order_relaxed) == 0) {
            int64_t zero = 0;
            oldest_ns.compare_exchange_strong(zero, now_ns());
        }
        before = queued_reqs.fetch_add((int64_t)ps.size());
        b0 = queued_bytes.fetch_add((int64_t)nbytes);
        const int64_t cap = cfg.max_batch_bytes;
        if (before <= 0 || (b0 < cap && b0 + (int64_t)nbytes >= cap)) {
            std::lock_guard<std::mutex> lk(mu);  // orders the wake-up after the builder's predicate check
            cv_submit.notify_one();
        }
        return first;
    }
}

// ---- builder ---------------------------------------------------------------
void cyaes_batcher::build_loop() {
    std::array<std::vector<Pend>, kShards> pend, spare;  // builder-private: taken, not yet batched
    std::array<size_t, kShards> ppos{};
    std::array<uint64_t, kShards> batched{};  // per shard: requests put into batches so far
    // (to, from, bytes) of the bounced requests' inputs; the workers run the
    // copies, so this is a plain local (a thread_local would be theirs, empty).
    std::vector<std::array<const uint8_t*, 3>> copies;
    int rr = 0;
    for (;;) {
        Stage* st = nullptr;
        const int64_t tw = now_ns();
        bool have = false;
        for (int s = 0; s < kShards && !have; s++) have = ppos[s] < pend[s].size();
        {
            std::unique_lock<std::mutex> lk(mu);
            if (!have && pending) {
                // The last batch's scatter rides on the next batch's move kernel;
                // with nothing queued for a short while (or a flush / stop), send
                // it alone.
                const auto until = Clock::now() + std::chrono::microseconds(std::min<uint32_t>(cfg.max_delay_us, 50));
                if (!cv_submit.wait_until(lk, until, [&] { return queued_reqs.load() > 0; }) || stop ||
                    flushers.load() > 0) {
                    if (queued_reqs.load() <= 0) {
                        lk.unlock();
                        flush_pending();
                        continue;
                    }
                }
            }
            if (!have) {
                cv_submit.wait(lk, [&] { return stop || queued_reqs.load() > 0; });
                if (queued_reqs.load() <= 0) break;  // stop requested and drained
                const int64_t t = oldest_ns.load();
                const auto due = Clock::time_point(std::chrono::nanoseconds(t ? t : now_ns())) +
                                 std::chrono::microseconds(cfg.max_delay_us);
                cv_submit.wait_until(lk, due, [&] {
                    return stop || flushers.load() > 0 || queued_bytes.load() >= (int64_t)cfg.max_batch_bytes;
                });
            }
            // Every other stage in flight has been handed to the completion
            // thread and will come back; only a lone pending stage must drain.
            if (free_stages.empty() && pending && stages.size() == 1) {
                lk.unlock();
                flush_pending();
                lk.lock();
            }
            cv_free.wait(lk, [&] { return !free_stages.empty(); });
            st = free_stages.back();
            free_stages.pop_back();
        }
        const int64_t tt = now_ns();
        pb.wait += tt - tw;
        oldest_ns.store(0);
        int64_t took = 0, took_bytes = 0;
        for (int s = 0; s < kShards; s++) {
            Shard& sh = shards[s];
            {
                std::lock_guard<std::mutex> lk(sh.mu);
                if (sh.q.empty()) continue;
                sh.q.swap(spare[s]);
                took_bytes += (int64_t)sh.bytes;
                sh.bytes = 0;
            }
            took += (int64_t)spare[s].size();
            if (ppos[s] == pend[s].size()) {
                pend[s].clear();
                ppos[s] = 0;
            }
            if (pend[s].empty()) pend[s].swap(spare[s]);
            else pend[s].insert(pend[s].end(), spare[s].begin(), spare[s].end());
            spare[s].clear();
        }
        queued_reqs.fetch_sub(took);
        queued_bytes.fetch_sub(took_bytes);
        const int64_t tl = now_ns();
        pb.take += tl - tt;

        // Lay the batch out: shards in rotating order, each shard's requests in
        // submission order, until the stage's requests, data or bounce is full.
        st->ne = st->nd = 0;
        st->emax = 0;
        st->dbytes = 0;
        st->bytes = 0;
        st->cbs.clear();
        st->segs.clear();
        st->bouts.clear();
        uint64_t data = 0, bounce = 0;
        bool full = false;
        copies.clear();
        for (int k = 0; k < kShards && !full; k++) {
            const int s = (rr + k) % kShards;
            std::vector<Pend>& q = pend[s];
            const uint32_t cb0 = (uint32_t)st->cbs.size();
            size_t i = ppos[s];
            for (; i < q.size(); i++) {
                Pend& p = q[i];
                const uint64_t sb = stage_bytes(p.d), bb = p.bounce ? bounce_bytes(p.d) : 0;
                // (the first request of a batch always fits: submit caps a request's size)
                if (st->ne + st->nd > 0 &&
                    (st->ne + st->nd == kMaxReqs || data + sb > data_cap || bounce + bb > bounce_cap)) {
                    full = true;
                    break;
                }
                BatchDesc d = p.d;
                d.stage = (uint32_t)data;
                data += sb;
                if (p.bounce) {  // through the pinned bounce buffer: in now, out at completion
                    uint8_t* hb = st->h_bounce + bounce;
                    const uint8_t* in = reinterpret_cast<const uint8_t*>((uintptr_t)p.d.src);
                    uint8_t* out = reinterpret_cast<uint8_t*>((uintptr_t)p.d.dst);
                    const uint32_t in_n = d.size;  // ENC/DEC data, SEAL chunk, OPEN packet
                    if (in_n) copies.push_back({hb, in, reinterpret_cast<const uint8_t*>((uintptr_t)in_n)});
                    d.src = d.dst = st->bounce_dev + bounce;
                    switch (d.op) {
                        case cyaes::kOpRelaySeal:
                            st->bouts.push_back({out, hb, CYAES_RELAY_PAYLOAD_OFFSET + d.crypt});
                            break;
                        case cyaes::kOpRelayOpen:
                            st->bouts.push_back({out + CYAES_RELAY_PAYLOAD_OFFSET, hb + CYAES_RELAY_PAYLOAD_OFFSET, d.crypt});
                            break;
                        default:
                            if (d.size) st->bouts.push_back({out, hb, d.size});
                    }
                    bounce += bb;
                }
                if (d.op == cyaes::kOpEncrypt || d.op == cyaes::kOpRelaySeal) {
                    st->h_enc[st->ne++] = d;
                    st->emax = std::max(st->emax, d.crypt);
                } else {
                    st->h_dec[st->nd++] = d;
                    st->dbytes += d.crypt;
                }
                st->cbs.push_back(p.cb);
                st->bytes += d.crypt;
            }
            const uint32_t taken = (uint32_t)(i - ppos[s]);
            if (taken) {
                batched[s] += taken;
                st->segs.push_back({(uint8_t)s, cb0, (uint32_t)st->cbs.size(), batched[s]});
            }
            ppos[s] = i;
        }
        rr = (rr + 1) % kShards;
        const int64_t tc = now_ns();
        pb.layout += tc - tl;
        if (st->cbs.empty()) {  // nothing taken (raced)
            std::lock_guard<std::mutex> lk(mu);
            free_stages.push_back(st);
            continue;
        }
        in_pool->run((copies.size() + kCopyChunk - 1) / kCopyChunk, [&](size_t c) {
            for (size_t i = c * kCopyChunk; i < std::min(copies.size(), (c + 1) * kCopyChunk); i++)
                memcpy(const_cast<uint8_t*>(copies[i][0]), copies[i][1], (size_t)(uintptr_t)copies[i][2]);
        });
        const int64_t ts = now_ns();
        pb.copy_in += ts - tc;
        st->status = launch(st);
        pb.submit += now_ns() - ts;
    }
    flush_pending();
    std::lock_guard<std::mutex> lk(mu);
    builder_done = true;
    cv_inflight.notify_all();
}

// To the completion thread, in launch order.
void cyaes_batcher::hand_off(Stage* st) {
    std::lock_guard<std::mutex> lk(mu);
    inflight.push_back(st);
    cv_inflight.notify_one();
}

// The pending batch's scatter on its own move kernel.
void cyaes_batcher::flush_pending() {
    Stage* p = pending;
    if (!p) return;
    pending = nullptr;
    if (p->status == CYAES_OK) {  // (a failed batch is not scattered: its outputs would be garbage)
        cyaes::BatchMove m{};
        m.sdesc = p->d_desc;
        m.sn = p->ne + p->nd;
        m.sstage = p->d_data;
        hipError_t e = cyaes::launch_batch_move(m, move_waves, pipe);
        if (e == hipSuccess) e = hipEventRecord(p->done, pipe);
        p->status = map_err(e);
    }
    hand_off(p);
}

// On the pipeline stream: H2D of the descriptors; one move kernel gathering
// this batch and scattering the pending one (whose completion event follows);
// then this batch's encrypt and decrypt kernels.  This batch becomes pending.
int cyaes_batcher::launch(Stage* st) {
    const uint32_t ne = st->ne, nd = st->nd, n = ne + nd;
    Stage* prev = pending;
    pending = nullptr;
    hipError_t e = hipSuccess;
    if (ne) e = hipMemcpyAsync(st->d_desc, st->h_enc, ne * sizeof(BatchDesc), hipMemcpyHostToDevice, pipe);
    if (e == hipSuccess && nd)
        e = hipMemcpyAsync(st->d_desc + ne, st->h_dec, nd * sizeof(BatchDesc), hipMemcpyHostToDevice, pipe);
    const bool sc = prev && prev->status == CYAES_OK;  // (a failed batch is not scattered)
    cyaes::BatchMove m{st->d_desc, n, sc ? prev->ne + prev->nd : 0u, st->d_data, st->d_offs, st->d_nb, st->d_kid,
                       sc ? prev->d_desc : nullptr, sc ? prev->d_data : nullptr};
    if (e == hipSuccess) e = cyaes::launch_batch_move(m, move_waves, pipe);
    if (prev) {
        if (sc && e == hipSuccess) e = hipEventRecord(prev->done, pipe);
        if (sc) prev->status = map_err(e);
        hand_off(prev);
    }
    int rc = map_err(e);
    // The batch's encrypt-type and decrypt-type lists: one after the other, or
    // side by side when the encrypt has long chains (relay chunks of >= 16 KiB:
    // its latency-bound chains leave most CUs to the decrypt).  dec_small: the
    // decrypt's full-chip time (~1.4 GB/ms) under a sixth of the longest
    // chain's (~0.6 us a block), too short to pay for a denser encrypt
    // (the runtime then keeps the two launches unless packing costs nothing).
    const double enc_us = st->emax / 16.0 * 0.6, dec_us = st->dbytes / 1.4e6;
    if (rc == CYAES_OK && ne && nd && st->emax >= kDuplexMinChain)
        rc = cyaes::ragged_duplex_batch(ctx, d_keys, key_cap, st->d_data, st->d_offs, st->d_nb, ne, st->d_kid,
                                        st->d_offs + ne, st->d_nb + ne, nd, st->d_kid + ne, pipe,
                                        dec_us * 6.0 < enc_us);
    else {
        if (rc == CYAES_OK && ne)
            rc = cyaes::ragged_batch(ctx, false, d_keys, key_cap, st->d_data, st->d_data, st->d_offs, st->d_nb, ne,
                                     st->d_kid, pipe);
        if (rc == CYAES_OK && nd)
            rc = cyaes::ragged_batch(ctx, true, d_keys, key_cap, st->d_data, st->d_data, st->d_offs + ne,
                                     st->d_nb + ne, nd, st->d_kid + ne, pipe);
    }
    pending = st;  // (a failed batch still goes through flush / the next launch, with its status)
    return rc;
}

// ---- completion ------------------------------------------------------------
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
        // A stage whose launch failed part-way may still have work in flight on
        // its buffers: drain the pipeline before the stage is reused.
        if (status != CYAES_OK) (void)hipStreamSynchronize(pipe);
        const int64_t t1 = now_ns();
        pc.sync += t1 - t0;
        if (status == CYAES_OK)
            workers->run((st->bouts.size() + kCopyChunk - 1) / kCopyChunk, [st](size_t c) {
                for (size_t i = c * kCopyChunk; i < std::min(st->bouts.size(), (c + 1) * kCopyChunk); i++)
                    memcpy(st->bouts[i].to, st->bouts[i].from, st->bouts[i].bytes);
            });
        const int64_t t2 = now_ns();
        pc.copy_out += t2 - t1;
        // The stage's outputs are out: hand it back to the builder now and run
        // its callbacks from completer-owned lists (swapped with last batch's,
        // so no allocation), so the GPU pipeline does not wait on callbacks.
        // Batches still complete one after another, so each shard's callbacks
        // keep their submission order.
        run_cbs.swap(st->cbs);
        run_segs.swap(st->segs);
        st->cbs.clear();
        st->segs.clear();
        const uint64_t sbytes = st->bytes;
        {
            std::lock_guard<std::mutex> g(mu);
            free_stages.push_back(st);
        }
        cv_free.notify_one();
        // Callbacks: one job per shard run, in that shard's submission order.
        // Poll mode: requests without a callback go to their shard's queue in
        // one locked append per run.
        const bool poll = (cfg.flags & CYAES_BATCHER_POLL) != 0;
        const std::vector<Cb>& cbs = run_cbs;
        const std::vector<Seg>& segs = run_segs;
        workers->run(segs.size(), [this, &cbs, &segs, status, poll](size_t k) {
            const Seg& g = segs[k];
            if (poll) {
                thread_local std::vector<Done> out;
                out.clear();
                for (uint32_t i = g.begin; i < g.end; i++) {
                    if (cbs[i].done) cbs[i].done(cbs[i].user, status);
                    else out.push_back({cbs[i].user, status});
                }
                if (!out.empty()) {
                    Shard& sh = shards[g.shard];
                    std::lock_guard<std::mutex> lk(sh.cmu);
                    sh.cq.insert(sh.cq.end(), out.begin(), out.end());
                }
                return;
            }
            for (uint32_t i = g.begin; i < g.end; i++)
                if (cbs[i].done) cbs[i].done(cbs[i].user, status);
        });
        const size_t nreq = cbs.size();
        pc.callbacks += now_ns() - t2;
        pc.batches++;
        pc.reqs += (int64_t)nreq;
        lk.lock();
        completed += nreq;
        for (const Seg& g : segs) done_seq[g.shard] = std::max(done_seq[g.shard], g.last_seq);
        batches++;
        bytes += sbytes;
        max_batch = std::max<uint64_t>(max_batch, nreq);
        if (status != CYAES_OK) {
            errors += nreq;
            if (first_error == CYAES_OK) first_error = status;
        }
        cv_flush.notify_all();
    }
}

// Waits until every shard has completed `target` requests; leaves first_error alone.
void cyaes_batcher::wait_done(const std::array<uint64_t, kShards>& target) {
    std::unique_lock<std::mutex> lk(mu);
    flushers.fetch_add(1);
    cv_submit.notify_all();
    cv_flush.wait(lk, [&] {
        for (int i = 0; i < kShards; i++)
            if (done_seq[i] < target[i]) return false;
        return true;
    });
    flushers.fetch_sub(1);
}

// Flush semantics: wait, then hand over (and clear) the first error since the previous flush.
int cyaes_batcher::wait_enqueued(const std::array<uint64_t, kShards>& target) {
    wait_done(target);
    std::lock_guard<std::mutex> lk(mu);
    const int err = first_error;
    first_error = CYAES_OK;
    return err;
}

static std::array<uint64_t, kShards> enqueue_counts(cyaes_batcher* b) {
    std::array<uint64_t, kShards> t;
    for (int i = 0; i < kShards; i++) {
        std::lock_guard<std::mutex> sl(b->shards[i].mu);
        t[i] = b->shards[i].enqueued;
    }
    return t;
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
    if (c.max_sessions == 0) c.max_sessions = 65536;
    if (c.max_batch_bytes < 4096 || c.max_batch_bytes > (1u << 30) || c.inflight > 16 || c.workers > 64 ||
        c.max_sessions > (1u << 22) || (c.flags & ~CYAES_BATCHER_POLL))
        return CYAES_EINVAL;
    cyaes_gpu* ctx = nullptr;
    int st = cyaes_gpu_create(c.device, &ctx);
    if (st) return st;
    auto* b = new cyaes_batcher();
    b->cfg = c;
    b->ctx = ctx;
    // HBM stage: max_batch_bytes of data, plus 16 B of relay header room per
    // request, rounded: the cut never lets a batch exceed it (a first request is
    // always taken; submit caps a request at max_batch_bytes).
    b->data_cap = (uint64_t)c.max_batch_bytes;
    b->bounce_cap = (uint64_t)c.max_batch_bytes + 2 * 65536;
    // Move-kernel waves (one request each at a time, split between the two
    // directions): enough packets in flight to cover PCIe latency both ways.
    b->move_waves = std::max(64, cyaes_gpu_num_cus(ctx) * 8);
    if (const char* w = getenv("CYAES_BATCH_COPY_WAVES")) b->move_waves = std::max(2, atoi(w));  // A/B
    b->key_cap = c.max_sessions;
    b->stages.resize(c.inflight);
    int dev_prev = 0;
    (void)hipGetDevice(&dev_prev);
    hipError_t e = hipSetDevice(c.device);
    const uint64_t data_room = b->data_cap + 16ull * kMaxReqs + 4096;
    for (Stage& s : b->stages) {
        const uint64_t meta = 2ull * kMaxReqs * sizeof(BatchDesc);
        uint8_t* h = nullptr;
        if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&h), meta, hipHostMallocDefault);
        if (e == hipSuccess) {
            s.h_enc = reinterpret_cast<BatchDesc*>(h);
            s.h_dec = s.h_enc + kMaxReqs;
            e = hipHostMalloc(reinterpret_cast<void**>(&s.h_bounce), b->bounce_cap, hipHostMallocMapped);
        }
        if (e == hipSuccess) {
            void* dp = nullptr;
            e = hipHostGetDevicePointer(&dp, s.h_bounce, 0);
            s.bounce_dev = (uint64_t)(uintptr_t)dp;
        }
        const uint64_t lists = (uint64_t)kMaxReqs * (sizeof(BatchDesc) + 8 + 4 + 4);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s.d_mem), lists + data_room);
        if (e == hipSuccess) {
            s.d_desc = reinterpret_cast<BatchDesc*>(s.d_mem);
            s.d_offs = reinterpret_cast<uint64_t*>(s.d_desc + kMaxReqs);
            s.d_nb = reinterpret_cast<uint32_t*>(s.d_offs + kMaxReqs);
            s.d_kid = s.d_nb + kMaxReqs;
            s.d_data = reinterpret_cast<uint8_t*>(s.d_kid + kMaxReqs);
        }
        if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
        s.cbs.reserve(kMaxReqs);
        b->free_stages.push_back(&s);
    }
    b->run_cbs.reserve(kMaxReqs);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&b->d_keys), (uint64_t)b->key_cap * kSchedBytes);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&b->pipe, hipStreamNonBlocking);
    (void)hipSetDevice(dev_prev);
    if (e != hipSuccess) {
        b->builder_done = true;
        cyaes_batcher_destroy(b);
        return map_err(e);
    }
    b->in_pool.reset(new Pool((int)c.workers - 1));  // + the builder thread itself
    b->workers.reset(new Pool((int)c.workers - 1));  // + the completion thread itself
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
                "[cyaes_batcher] %lld batches, %.0f reqs/batch; per batch (us): builder wait %.0f take %.0f layout "
                "%.0f copy-in %.0f submit %.0f | completer sync %.0f copy-out %.0f callbacks %.0f\n",
                (long long)C.batches, C.reqs / nb, B.wait * us / nb, B.take * us / nb, B.layout * us / nb,
                B.copy_in * us / nb, B.submit * us / nb, C.sync * us / nb, C.copy_out * us / nb, C.callbacks * us / nb);
    }
    b->workers.reset();
    b->in_pool.reset();
    int dev_prev = 0;
    (void)hipGetDevice(&dev_prev);
    (void)hipSetDevice(b->cfg.device);
    if (b->pipe) (void)hipStreamSynchronize(b->pipe);
    for (Stage& s : b->stages) {
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.d_mem) (void)hipFree(s.d_mem);
        if (s.h_enc) (void)hipHostFree(s.h_enc);
        if (s.h_bounce) (void)hipHostFree(s.h_bounce);
    }
    if (b->d_keys) (void)hipFree(b->d_keys);
    if (b->pipe) (void)hipStreamDestroy(b->pipe);
    for (cyaes::PinHold& h : b->pool_pins) (void)cyaes::pin_release(&h);  // pools the caller left registered
    (void)hipSetDevice(dev_prev);
    (void)cyaes_gpu_destroy(b->ctx);
    delete b;
}

int cyaes_batcher_session_open(cyaes_batcher* b, const uint8_t key[16], uint32_t* slot) {
    if (!b || !key || !slot) return CYAES_EINVAL;
    cyaes_key k;
    cyaes::expand_key(key, &k);
    uint32_t sched[cyaes::kSchedWords];
    cyaes::to_device_schedule(k, sched);
    std::lock_guard<std::mutex> lk(b->smu);
    // Rows retired by closes whose earlier requests have all completed are free again.
    if (!b->retired.empty()) {
        std::array<uint64_t, kShards> done;
        {
            std::lock_guard<std::mutex> l2(b->mu);
            done = b->done_seq;
        }
        auto it = std::remove_if(b->retired.begin(), b->retired.end(), [&](const cyaes_batcher::Retired& r) {
            for (int i = 0; i < kShards; i++)
                if (done[i] < r.stamp[i]) return false;
            b->free_rows.push_back(r.row);
            return true;
        });
        b->retired.erase(it, b->retired.end());
    }
    uint32_t row;
    if (!b->free_rows.empty()) {
        row = b->free_rows.back();
        b->free_rows.pop_back();
    } else if (b->next_row < b->key_cap) {
        row = b->next_row++;
    } else {
        return CYAES_ERANGE;  // max_sessions rows in use (or still referenced by queued requests)
    }
    int dev_prev = 0;
    (void)hipGetDevice(&dev_prev);
    (void)hipSetDevice(b->cfg.device);
    // Synchronous: every batch built after this returns sees the row.
    const hipError_t e = hipMemcpy(reinterpret_cast<uint8_t*>(b->d_keys) + (uint64_t)row * kSchedBytes, sched,
                                   kSchedBytes, hipMemcpyHostToDevice);
    (void)hipSetDevice(dev_prev);
    if (e != hipSuccess) {
        b->free_rows.push_back(row);
        return map_err(e);
    }
    size_t i = 0;
    while (i < b->slot_row.size() && b->slot_row[i] != kNoRow) i++;
    if (i == b->slot_row.size()) b->slot_row.push_back(kNoRow);
    b->slot_row[i] = row;
    b->sessions_version.fetch_add(1, std::memory_order_release);
    *slot = (uint32_t)i;
    return CYAES_OK;
}

int cyaes_batcher_session_close(cyaes_batcher* b, uint32_t slot) {
    if (!b) return CYAES_EINVAL;
    std::lock_guard<std::mutex> lk(b->smu);
    if (slot >= b->slot_row.size() || b->slot_row[slot] == kNoRow) return CYAES_ERANGE;
    const uint32_t row = b->slot_row[slot];
    b->slot_row[slot] = kNoRow;
    b->sessions_version.fetch_add(1, std::memory_order_release);
    // Stamp after the version bump: a request enqueued later sees the new version.
    b->retired.push_back({row, enqueue_counts(b)});
    return CYAES_OK;
}

int cyaes_batcher_register_pool(cyaes_batcher* b, void* base, size_t bytes, uint32_t* pool) {
    if (!b || !base || !bytes || !pool || (uintptr_t)base + bytes < (uintptr_t)base) return CYAES_EINVAL;
    std::lock_guard<std::mutex> lk(b->pmu);
    int slot = -1;
    for (int i = 0; i < kMaxPools; i++) {
        const PoolEnt& e = b->pools[i];
        if (e.live && (uintptr_t)base < (uintptr_t)e.host + e.bytes && (uintptr_t)e.host < (uintptr_t)base + bytes)
            return CYAES_EINVAL;  // overlaps a registered pool
        if (!e.live && slot < 0) slot = i;
    }
    if (slot < 0) return CYAES_ENOMEM;
    int dev_prev = 0;
    (void)hipGetDevice(&dev_prev);
    (void)hipSetDevice(b->cfg.device);
    // The pool's exact bytes (the caller's buffer need not be page aligned):
    // the registry registers the whole pages they cover, shared with other
    // pools' registrations on the same pages, and tests a foreign registration
    // on the bytes themselves.
    cyaes::PinHold held;
    int st = cyaes::pin_acquire((uintptr_t)base, (uintptr_t)base + bytes, cyaes::PinMode::kShared, &held);
    if (st == cyaes::kPinConflict) st = CYAES_EINVAL;  // part of the pages registered by another owner
    // The device view must be one contiguous range: check it at the end and at
    // every boundary between the registrations that hold the pool.
    void* dev = nullptr;
    if (st == CYAES_OK && hipHostGetDevicePointer(&dev, base, 0) != hipSuccess) st = CYAES_EINVAL;
    if (st == CYAES_OK) {
        std::vector<uintptr_t> probe{(uintptr_t)base + bytes - 1}, bounds;
        cyaes::pin_bounds(held, &bounds);
        for (size_t i = 0; i < bounds.size(); i += 2)
            for (uintptr_t q : {bounds[i], bounds[i + 1] - 1, bounds[i + 1]})
                if (q > (uintptr_t)base && q < (uintptr_t)base + bytes) probe.push_back(q);
        for (uintptr_t q : probe) {
            void* dq = nullptr;
            if (hipHostGetDevicePointer(&dq, reinterpret_cast<void*>(q), 0) != hipSuccess ||
                (uintptr_t)dq - (uintptr_t)dev != q - (uintptr_t)base) {
                st = CYAES_EINVAL;
                break;
            }
        }
    }
    if (st != CYAES_OK) {
        (void)cyaes::pin_release(&held);
        (void)hipGetLastError();
        (void)hipSetDevice(dev_prev);
        return st;
    }
    (void)hipSetDevice(dev_prev);
    b->pools[slot] = PoolEnt{static_cast<uint8_t*>(base), (uint64_t)(uintptr_t)dev, (uint64_t)bytes, true};
    b->pool_pins[slot] = std::move(held);
    b->pools_version.fetch_add(1, std::memory_order_release);
    *pool = (uint32_t)slot;
    return CYAES_OK;
}

int cyaes_batcher_unregister_pool(cyaes_batcher* b, uint32_t pool) {
    if (!b || pool >= (uint32_t)kMaxPools) return CYAES_EINVAL;
    cyaes::PinHold held;  // its references stay taken until the requests below are done
    {
        std::lock_guard<std::mutex> lk(b->pmu);
        if (!b->pools[pool].live) return CYAES_EINVAL;
        b->pools[pool].live = false;
        std::swap(held, b->pool_pins[pool]);
        b->pools_version.fetch_add(1, std::memory_order_release);
    }
    // Requests enqueued before the removal may still read or write the pool.
    // Their errors stay for the next cyaes_batcher_flush (cyaes_batch.h).
    b->wait_done(enqueue_counts(b));
    std::lock_guard<std::mutex> lk(b->pmu);
    int dev_prev = 0;
    (void)hipGetDevice(&dev_prev);
    (void)hipSetDevice(b->cfg.device);
    const int st = cyaes::pin_release(&held);  // pages another live pool still uses stay registered
    (void)hipSetDevice(dev_prev);
    return st;
}

int cyaes_batcher_submit_many(cyaes_batcher* b, const cyaes_batch_req* reqs, uint32_t n, int* status) {
    if (!b || (n && !reqs)) return CYAES_EINVAL;
    if (b->stop.load()) return CYAES_EINVAL;
    return b->enqueue([&](const Snap& ss, std::vector<Pend>& ps, uint64_t& nbytes) {
        int first = CYAES_OK;
        ps.resize(n);
        size_t k = 0;
        for (uint32_t i = 0; i < n; i++) {
            const int st = b->make(reqs[i], ss, &ps[k]);
            if (status) status[i] = st;
            if (st) {
                if (first == CYAES_OK) first = st;
                continue;
            }
            nbytes += stage_bytes(ps[k].d);
            k++;
        }
        ps.resize(k);
        return first;
    });
}

int cyaes_batcher_submit_pooled(cyaes_batcher* b, const cyaes_pool_req* reqs, uint32_t n, int* status) {
    if (!b || (n && !reqs)) return CYAES_EINVAL;
    if (b->stop.load()) return CYAES_EINVAL;
    return b->enqueue([&](const Snap& ss, std::vector<Pend>& ps, uint64_t& nbytes) {
        int first = CYAES_OK;
        ps.resize(n);
        size_t k = 0;
        for (uint32_t i = 0; i < n; i++) {
            const int st = b->make_pooled(reqs[i], ss, &ps[k]);
            if (status) status[i] = st;
            if (st) {
                if (first == CYAES_OK) first = st;
                continue;
            }
            nbytes += stage_bytes(ps[k].d);
            k++;
        }
        ps.resize(k);
        return first;
    });
}

int cyaes_batcher_submit(cyaes_batcher* b, int op, uint32_t slot, const uint8_t* in, uint8_t* out, size_t size,
                         cyaes_done_fn done, void* user) {
    if (!b || (op != CYAES_OP_ENCRYPT && op != CYAES_OP_DECRYPT) || size > 0xFFFFFFFFu) return CYAES_EINVAL;
    const cyaes_batch_req q{op, slot, 0, in, out, (uint32_t)size, done, user};
    int st = CYAES_OK;
    const int rc = cyaes_batcher_submit_many(b, &q, 1, &st);
    return rc ? rc : st;
}

int cyaes_batcher_submit_seal(cyaes_batcher* b, uint32_t slot, int32_t conn_id, const uint8_t* payload,
                              uint32_t size, uint8_t* packet_out, cyaes_done_fn done, void* user) {
    if (!b) return CYAES_EINVAL;
    const cyaes_batch_req q{CYAES_OP_RELAY_SEAL, slot, conn_id, payload, packet_out, size, done, user};
    int st = CYAES_OK;
    const int rc = cyaes_batcher_submit_many(b, &q, 1, &st);
    return rc ? rc : st;
}

int cyaes_batcher_submit_open(cyaes_batcher* b, uint32_t slot, uint8_t* packet, uint32_t packet_bytes,
                              cyaes_done_fn done, void* user) {
    if (!b) return CYAES_EINVAL;
    const cyaes_batch_req q{CYAES_OP_RELAY_OPEN, slot, 0, packet, packet, packet_bytes, done, user};
    int st = CYAES_OK;
    const int rc = cyaes_batcher_submit_many(b, &q, 1, &st);
    return rc ? rc : st;
}

uint32_t cyaes_batcher_poll(cyaes_batcher* b, void** users, int* status, uint32_t max) {
    if (!b || !users || max == 0) return 0;
    Shard& sh = b->shards[my_shard()];
    std::lock_guard<std::mutex> lk(sh.cmu);
    const uint32_t n = (uint32_t)std::min<size_t>(max, sh.cq.size());
    for (uint32_t i = 0; i < n; i++) {
        users[i] = sh.cq[i].user;
        if (status) status[i] = sh.cq[i].status;
    }
    sh.cq.erase(sh.cq.begin(), sh.cq.begin() + n);
    return n;
}

int cyaes_batcher_flush(cyaes_batcher* b) {
    if (!b) return CYAES_EINVAL;
    return b->wait_enqueued(enqueue_counts(b));
}

int cyaes_batcher_stats(cyaes_batcher* b, uint64_t out[6]) {
    if (!b || !out) return CYAES_EINVAL;
    const std::array<uint64_t, kShards> enq = enqueue_counts(b);
    std::lock_guard<std::mutex> lk(b->mu);
    uint64_t total = 0;
    for (uint64_t v : enq) total += v;
    out[0] = b->completed;
    out[1] = b->batches;
    out[2] = b->bytes;
    out[3] = b->max_batch;
    out[4] = b->errors;
    out[5] = total >= b->completed ? total - b->completed : 0;
    return CYAES_OK;
}

}  // extern "C"
