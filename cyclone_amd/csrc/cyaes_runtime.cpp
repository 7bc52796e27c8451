// cyaes_runtime.cpp -- host runtime behind include/cyaes.h: device context,
// key table, batch launch geometry, host-memory drop-in path.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <new>
#include <vector>

#include "cyaes.h"
#include "cyaes_internal.h"
#include "cyaes_tables.h"

using namespace cyaes;

struct cyaes_gpu {
    int device = 0;
    int num_cus = 0;
    uint64_t quad_max_chains = CYAES_QUAD_MAX_CHAINS;  // env CYAES_QUAD_MAX_CHAINS (A/B only)
    uint32_t ragged_group = 0;  // env CYAES_RAGGED_GROUP: payloads per ragged-decrypt wave group (0 = auto; tests, A/B)
    uint32_t enc_run = 0;       // env CYAES_ENC_RUN: payloads per lane run of the uniform encrypt (0 = auto; tests, A/B)
    bool enc_no_sess = false;   // env CYAES_ENC_NO_SESS=1: keyed uniform encrypt always by waterfall (tests, A/B)
    bool enc_no_lines = false;  // env CYAES_ENC_LINES=0: strided encrypts without k_encrypt_lines (tests, A/B)
    bool enc_no_rag_lines = false;  // env CYAES_ENC_RAG_LINES=0: ragged encrypts without k_encrypt_rag_lines (tests, A/B)
    int lines_grid = 0;         // env CYAES_LINES_GRID: cap on k_encrypt_lines' grid (tests: several items per wave)
    int dec_dyn = -1;           // env CYAES_DEC_DYN: 1 / 0 force the dynamic decrypt pool on / off; -1: long launches only
    uint32_t dec_range_steps = kDecRangeSteps;  // env CYAES_DEC_RANGE_STEPS: steps per dynamic flat-decrypt range
    uint32_t dec_groups_per_wave = kDecGroupsPerWave;  // env CYAES_DEC_GROUPS_PER_WAVE: ragged groups per wave
    uint32_t dec_dyn_pct = kDecDynPct;  // env CYAES_DEC_DYN_PCT: % of a decrypt's work in the dynamic pool
    float dec_xcd_w[kXcds] = {};  // env CYAES_DEC_XCD_W=w0,...,w7: XCD-weighted static decrypt split (A/B; all 0: off)
    int dec_grid_max = 0;       // env CYAES_DEC_GRID: cap on decrypt workgroups (tests: many ranges per wave on small batches)
    bool strided_lists = false; // env CYAES_STRIDED_LISTS=1: strided decrypts as ragged batches (tests, A/B)
    bool strided_force = false; // env CYAES_STRIDED_FORCE=1: contiguous strided batches keep the strided kernels (A/B)
    bool dec_handoff = true;    // env CYAES_DEC_HANDOFF=0: in-place static decrypts snapshot their carries in a prepass
    bool duplex_off = false;    // env CYAES_DUPLEX=0: duplex calls run as two launches (tests, A/B)
    int duplex_pack = 12;       // env CYAES_DUPLEX_PACK: waves per workgroup of cyaes_gpu_duplex_ragged's encrypt (A/B)
    int dup_min_dec_wgs = 8;    // env CYAES_DUPLEX_DEC_WGS: least decrypt workgroups beside it (A/B)
    uint32_t duplex_dyn_pct = kDuplexDynPct;  // env CYAES_DUPLEX_DYN_PCT: the duplex decrypt's pool share (%)
    uint32_t* d_tables = nullptr;  // enc[512] | dec[512] | sbox[256 B]
    uint32_t* d_keys = nullptr;    // nkeys * kSchedWords
    uint32_t nkeys = 0;
    uint32_t key_cap = 0;
    uint32_t* d_status = nullptr;
    unsigned long long* d_digest = nullptr;
    struct HostPipe* pipe = nullptr;  // cyaes_gpu_{en,de}crypt_host, created on first use
    // Per-call scratch blocks (StreamScratch), cached for the context's life.
    struct ScratchBlock {
        void* p;
        uint64_t bytes;
        hipEvent_t done;     // recorded on the last user's stream behind its kernels
        hipStream_t stream;  // that stream
        bool in_use;         // held by a call that is still enqueuing
        bool pending;        // `done` recorded and not yet seen complete
    };
    std::mutex scratch_mu;
    std::vector<ScratchBlock> scratch;
    uint64_t scratch_bytes = 0;  // cached in `scratch`
    // Key table (d_keys) users: per stream that ran a batch reading it, an event
    // recorded behind that batch's kernels, so a write of the table waits for
    // exactly those streams, not for the device.
    std::mutex key_mu;
    std::vector<std::pair<hipStream_t, hipEvent_t>> key_uses;
    hipEvent_t keys_written = nullptr;    // behind cyaes_gpu_set_keys_device's expansion on the caller's stream
    bool keys_written_pending = false;
    std::vector<uint32_t*> retired_keys;  // tables outgrown while batches may still read them; freed at destroy
    // cyaes_gpu_duplex_ragged's second stream (created on first use: a
    // context-lifetime stream takes a hardware queue)
    std::mutex side_mu;
    hipStream_t side = nullptr;
};

namespace {


int map_err(hipError_t e) {
    if (e == hipSuccess) return CYAES_OK;
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return CYAES_ENOMEM;
    return CYAES_EDEVICE;
}

// Makes ctx->device current for the duration of a call, restoring the
// caller's device afterwards.
struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

#define CY_TRY(expr)                         \
    do {                                     \
        hipError_t _e = (expr);              \
        if (_e != hipSuccess) return map_err(_e); \
    } while (0)

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }


// Validates the key-selection arguments of a batch and fills a KeySel.  The
// key table is the context's, unless a batch brings its own (table != NULL:
// the drop-in's per-call schedule, the batcher's per-batch session keys).
int make_keysel(const cyaes_gpu* ctx, uint64_t npayloads, const uint32_t* key_idx, uint32_t ppk, KeySel* ks,
                const uint32_t* table = nullptr, uint32_t table_keys = 0) {
    const uint32_t nkeys = table ? table_keys : ctx->nkeys;
    if (nkeys == 0) return CYAES_ERANGE;
    if ((key_idx || ppk) && npayloads > 0xFFFFFFFFull) return CYAES_EINVAL;
    if (!key_idx && ppk && npayloads && (npayloads - 1) / ppk >= nkeys) return CYAES_ERANGE;
    ks->table = table ? table : ctx->d_keys;
    ks->key_idx = key_idx;
    ks->ppk = key_idx ? make_fastdiv(0) : make_fastdiv(ppk);
    ks->nkeys = nkeys;
    return CYAES_OK;
}

// A batch that read the context's key table was launched on `stream`.
bool reads_ctx_keys(const cyaes_gpu* ctx, const uint32_t* table) {
    return ctx->d_keys && table >= ctx->d_keys && table < ctx->d_keys + (uint64_t)ctx->key_cap * kSchedWords;
}
// Entries whose batches have completed are dropped on the way (r06, ADVICE
// r05): the list holds only streams with a table reader still in flight, so a
// caller that uses a new stream per request does not grow it, and a key write
// waits for at most that many events.
int note_key_use(cyaes_gpu* ctx, const uint32_t* table, hipStream_t stream) {
    if (!reads_ctx_keys(ctx, table)) return CYAES_OK;
    std::lock_guard<std::mutex> lk(ctx->key_mu);
    auto& v = ctx->key_uses;
    for (size_t i = 0; i < v.size();) {
        if (v[i].first == stream) return map_err(hipEventRecord(v[i].second, stream));
        const hipError_t q = hipEventQuery(v[i].second);
        if (q == hipSuccess) {
            (void)hipEventDestroy(v[i].second);
            v[i] = v.back();
            v.pop_back();
            continue;
        }
        if (q != hipErrorNotReady) return map_err(q);
        i++;
    }
    hipEvent_t ev = nullptr;
    CY_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    ctx->key_uses.push_back({stream, ev});
    return map_err(hipEventRecord(ev, stream));
}

constexpr uint64_t kRunMax = 8;               // payloads per encrypt run
constexpr uint32_t kRunMaxPayload = 8192;      // runs only for payloads up to 512 blocks

int enc_grid_cap(const cyaes_gpu* ctx) { return std::max(1, ctx->num_cus * kEncWgPerCu); }
int dec_grid_cap(const cyaes_gpu* ctx) {
    const int cap = std::max(1, ctx->num_cus * kDecWgPerCu);
    return ctx->dec_grid_max > 0 ? std::min(cap, ctx->dec_grid_max) : cap;
}

// Launch shape for `waves` independent wave-sized work items (encrypt: 64
// chains; ragged decrypt: one payload).  Enough to fill every CU with 16
// waves: full 1024-thread workgroups, grid capped at one per CU (persistent).
// Fewer: spread them, ceil(waves / CUs) waves per workgroup, so a small
// batch of serial chains runs on many CUs' LDS instead of queueing on one.
struct Shape {
    int grid, threads;
};
Shape wave_shape(const cyaes_gpu* ctx, uint64_t waves, int max_threads) {
    const uint64_t cus = (uint64_t)std::max(1, ctx->num_cus);
    const uint64_t per_wg = (uint64_t)max_threads / 64;
    if (waves >= cus * per_wg) return {(int)cus, max_threads};
    const uint64_t w = std::max<uint64_t>(1, (waves + cus - 1) / cus);
    return {(int)std::max<uint64_t>(1, (waves + w - 1) / w), (int)(64 * w)};
}

}  // namespace

// cyaes_gpu_duplex_ragged's packed encrypt: workgroups of about duplex_pack
// waves, their count a multiple of the shader engines (32: workgroups go to
// the XCDs in turn and to an XCD's four engines in turn, so the decrypt
// beside it finds the same number of free CUs on every engine).
constexpr int kDupUnit = 4 * (int)kXcds;
static int packed_enc_wgs(const cyaes_gpu* ctx, uint64_t npayloads) {
    const uint64_t qwaves = (4 * npayloads + 63) / 64, pw = (uint64_t)ctx->duplex_pack;
    const uint64_t e = ((qwaves + pw - 1) / pw + kDupUnit - 1) / kDupUnit * kDupUnit;
    return (int)std::min<uint64_t>(e, (uint64_t)std::max(kDupUnit, ctx->num_cus - kDupUnit));
}

bool cyaes::ragged_encrypt_is_quad(const cyaes_gpu* ctx, uint64_t n) {
    const uint64_t q = ctx->quad_max_chains;
    return n < (q > UINT64_MAX / kQuadRaggedFactor ? UINT64_MAX : q * kQuadRaggedFactor);
}

namespace {

// offsets == nullptr and stride != 0: a strided batch (payload p at off0 + p *
// stride, payload_bytes each), run by the ragged kernels without lists.
// An encrypt batch's arguments and launch shape (encrypt_common launches it;
// the duplex launch runs its lane walk inside the duplex grid).
struct EncPlan {
    EncArgs a;
    bool quad;     // k_encrypt_quad (latency-bound batch or small ragged one)
    bool sess;     // SESS grid: a lane per work item, not persistent
    int grid, threads;
};

int enc_plan(cyaes_gpu* ctx, const uint8_t* in, uint8_t* out, const uint64_t* offsets, const uint32_t* nbytes,
             uint64_t npayloads, uint32_t payload_bytes, const uint32_t* key_idx, uint32_t ppk, const uint8_t* iv_in,
             uint8_t* iv_out, const uint32_t* table, uint32_t table_keys, uint64_t off0, uint64_t stride,
             EncPlan* plan, bool pack = false) {
    EncArgs& a = plan->a;
    a = EncArgs{};
    plan->quad = plan->sess = false;
    a.off0 = off0;
    a.stride = stride;
    const bool ragged = offsets != nullptr || stride != 0;
    int st = make_keysel(ctx, npayloads, key_idx, ppk, &a.keys, table, table_keys);
    if (st) return st;
    a.in = in;
    a.out = out;
    a.offsets = offsets;
    a.nbytes = nbytes;
    a.npayloads = npayloads;
    a.payload_bytes = payload_bytes;
    a.iv_in = iv_in;
    a.iv_out = iv_out;
    a.tables = ctx->d_tables + kEncTableOff / 4;
    a.status = ctx->d_status;
    if (ragged ? ragged_encrypt_is_quad(ctx, npayloads) : npayloads < ctx->quad_max_chains) {
        // Latency-bound batch (fewer chains than lanes to fill the chip four
        // times over), or a ragged one: four lanes per chain (k_encrypt_quad).
        // pack (cyaes_gpu_duplex_ragged): ~12 waves per workgroup, on as few CUs
        // as hold them, leaving the rest of the chip to a concurrent launch.
        const uint64_t qwaves = (4 * npayloads + 63) / 64;
        Shape sh;
        if (pack) {
            const uint64_t e = (uint64_t)packed_enc_wgs(ctx, npayloads);
            sh = Shape{(int)e, (int)(64 * std::min<uint64_t>(16, (qwaves + e - 1) / e))};
        } else {
            sh = wave_shape(ctx, qwaves, kEncThreads);
        }
        plan->quad = true;
        plan->grid = std::min(sh.grid, enc_grid_cap(ctx));
        plan->threads = sh.threads;
        return CYAES_OK;
    }
    // Runs (k_encrypt RUNS): a uniform batch of short payloads with more
    // payloads than the chip has lanes gives each lane R consecutive payloads
    // as one block stream (contiguous, so the chunk prefetch never stops at a
    // payload start), with R payloads per lane-chain still leaving >= one work
    // item per lane; sessions must hold whole runs.
    // (With per-session keys on the waterfall path (config D) runs measured 3 %
    // slower, without keys (config B) 1.5 % faster, profiles/r03/ab_enc_runs.txt;
    // whole-wave sessions take the SESS path below, which has no waterfall.)
    const bool runs_ok = !ragged && !iv_in && !iv_out && !key_idx && payload_bytes <= kRunMaxPayload;
    const bool runs_auto = runs_ok;
    uint64_t R = 1;
    if (runs_auto) {
        const uint64_t lanes = (uint64_t)std::max(1, ctx->num_cus) * kEncThreads;
        R = std::max<uint64_t>(1, std::min<uint64_t>(kRunMax, npayloads / lanes));
        while (R > 1 && ppk % R) R--;
    }
    if (ctx->enc_run) R = ctx->enc_run;  // A/B override (env CYAES_ENC_RUN)
    if (!runs_ok || R == 0 || (ppk && ppk % R)) R = 1;
    // Sessions of payloads_per_key payloads that hold whole waves of work items
    // (64 lanes x R payloads; config D: 256 = 64 x 4): the key is per wave
    // (SESS).  Otherwise keyed batches take the per-lane waterfall, without runs
    // unless forced.
    bool sess = false;
    if (!ragged && !key_idx && ppk && !ctx->enc_no_sess) {
        uint64_t r = R;
        while (r > 1 && ppk % (64 * r)) r--;
        if (ppk % (64 * r) == 0) {
            sess = true;
            R = r;
        }
    }
    if (ppk && !sess && !ctx->enc_run) R = 1;
    a.run = (uint32_t)R;
    a.sess_payloads = sess ? ppk : 0;
    const uint64_t waves = ((npayloads + a.run - 1) / a.run + 63) / 64;
    const Shape sh = wave_shape(ctx, waves, kEncThreads);
    // SESS: one pass, a lane per work item (the kernel loads each wave's
    // schedule once, before its loop); more workgroups than CUs queue.
    const uint64_t sess_grid = (waves * 64 + sh.threads - 1) / sh.threads;
    if (sess && sess_grid > (uint64_t)INT32_MAX) return CYAES_EINVAL;
    plan->sess = sess;
    plan->grid = sess ? (int)sess_grid : std::min(sh.grid, enc_grid_cap(ctx));
    plan->threads = sh.threads;
    return CYAES_OK;
}

int encrypt_rag_lines(cyaes_gpu* ctx, const EncArgs& a, uint64_t nrag, hipStream_t stream);

int encrypt_common(cyaes_gpu* ctx, const uint8_t* in, uint8_t* out, const uint64_t* offsets, const uint32_t* nbytes,
                   uint64_t npayloads, uint32_t payload_bytes, const uint32_t* key_idx, uint32_t ppk,
                   const uint8_t* iv_in, uint8_t* iv_out, hipStream_t stream, const uint32_t* table = nullptr,
                   uint32_t table_keys = 0, uint64_t off0 = 0, uint64_t stride = 0, bool pack = false) {
    EncPlan plan;
    int st = enc_plan(ctx, in, out, offsets, nbytes, npayloads, payload_bytes, key_idx, ppk, iv_in, iv_out, table,
                      table_keys, off0, stride, &plan, pack);
    if (st) return st;
    // A strided batch for the lane kernel, unkeyed and without IV arrays: its
    // whole 1,024-payload groups are read by 64-B lines (k_encrypt_lines), the
    // rest (if any) by the ordinary plan.
    // The kernel's offsets from the stream base are 32-bit (lines reach <= 63 B past a payload).
    const uint64_t nlines_pay = npayloads / kLinesGroup * kLinesGroup;
    const bool span32 = nlines_pay && (nlines_pay - 1) * stride + payload_bytes + off0 + 64 <= 0xFFFFFFFFull;
    if (stride && !offsets && !key_idx && !ppk && !iv_in && !iv_out && !plan.quad && span32 && !ctx->enc_no_lines) {
        EncArgs la = plan.a;
        la.npayloads = nlines_pay;
        const Shape sh = wave_shape(ctx, nlines_pay / 64, kEncThreads);
        int grid = std::min(sh.grid, enc_grid_cap(ctx));
        if (ctx->lines_grid > 0) grid = std::min(grid, ctx->lines_grid);
        CY_TRY(launch_encrypt_lines(la, grid, sh.threads, stream));
        st = note_key_use(ctx, la.keys.table, stream);
        if (st || nlines_pay == npayloads) return st;
        return encrypt_common(ctx, in, out, nullptr, nullptr, npayloads - nlines_pay, payload_bytes, nullptr, 0,
                              nullptr, nullptr, stream, table, table_keys, off0 + nlines_pay * stride, stride);
    }
    // A ragged (list) batch for the lane kernel, unkeyed and without IV arrays:
    // its whole 1,024-payload groups by lines first (encrypt_rag_lines).
    const uint64_t nrag = npayloads / kLinesGroup * kLinesGroup;
    if (offsets && !stride && !key_idx && !ppk && !iv_in && !iv_out && !plan.quad && nrag && !ctx->enc_no_lines &&
        !ctx->enc_no_rag_lines) {
        st = encrypt_rag_lines(ctx, plan.a, nrag, stream);
        if (st || nrag == npayloads) return st;
        return encrypt_common(ctx, in, out, offsets + nrag, nbytes + nrag, npayloads - nrag, payload_bytes, nullptr, 0,
                              nullptr, nullptr, stream, table, table_keys);
    }
    if (plan.quad) CY_TRY(launch_encrypt_quad(plan.a, plan.grid, plan.threads, stream));
    else CY_TRY(launch_encrypt(plan.a, plan.grid, plan.threads, stream));
    return note_key_use(ctx, plan.a.keys.table, stream);
}

// Per-call device scratch (the decrypt's work words and range-boundary
// snapshots, IV copies, strided lists), stream-ordered by events: blocks come
// from hipMalloc and stay cached in the context; releasing one records an
// event on the batch's stream behind the kernels that use it, and a block is
// handed out again only once its event has completed.  So batches of one
// context on different streams never share a block while a kernel still
// reads it, and nothing is freed before the context is destroyed.
// (Until late r04 the blocks came from a private hipMemPool.  r04 blamed that
// pool for two illegal-address reports on torch host-to-device copies; r05
// traced them to host registrations instead (a registration that outlives
// its memory).  The plain hipMalloc blocks stayed.)
constexpr size_t kScratchMaxBlocks = 64;             // beyond this, reuse a pending block behind its event
constexpr uint64_t kScratchCacheBytes = 256ull << 20;  // above this, completed blocks are freed, largest first

struct StreamScratch {
    void* p = nullptr;
    cyaes_gpu* ctx = nullptr;
    size_t idx = 0;
    hipStream_t s = nullptr;
    int get(cyaes_gpu* c, uint64_t bytes, hipStream_t stream) {
        std::vector<ScratchVictim> victims;
        uint64_t cap = 0;
        const int st = pick(c, bytes, stream, &victims, &cap);
        // hipFree and hipMalloc may wait for the device: never under the
        // mutex, so a new block is made after it is released.
        for (const auto& x : victims) {
            (void)hipFree(x.first);
            (void)hipEventDestroy(x.second);
        }
        if (st || p) return st;
        void* mem = nullptr;
        hipEvent_t ev = nullptr;
        hipError_t e = hipMalloc(&mem, cap);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        std::lock_guard<std::mutex> lk(c->scratch_mu);
        if (e != hipSuccess) {
            if (mem) (void)hipFree(mem);
            c->scratch_bytes -= cap;  // (reserved by pick)
            return map_err(e);
        }
        auto& v = c->scratch;
        size_t slot = 0;  // an empty slot, else a new one
        while (slot < v.size() && v[slot].p) slot++;
        if (slot == v.size()) v.push_back({});
        v[slot] = {mem, cap, ev, stream, true, false};
        p = mem;
        ctx = c;
        idx = slot;
        s = stream;
        return CYAES_OK;
    }
    using ScratchVictim = std::pair<void*, hipEvent_t>;
    // Under the mutex: hands out a cached block (p set), or reserves `cap`
    // bytes for a new one and takes out the completed blocks trim() frees.
    int pick(cyaes_gpu* c, uint64_t bytes, hipStream_t stream, std::vector<ScratchVictim>* victims, uint64_t* cap_out) {
        std::lock_guard<std::mutex> lk(c->scratch_mu);
        auto& v = c->scratch;
        // Preference: a completed block, or one whose last user was this very
        // stream (stream order already puts this call behind it), smallest
        // first; else, at the block limit, a pending block of another stream,
        // which this stream then waits for on the device (never
        // block the host under the mutex).
        size_t best = v.size(), other = v.size();
        for (size_t i = 0; i < v.size(); i++) {
            auto& b = v[i];
            if (!b.p || b.in_use || b.bytes < bytes) continue;
            if (b.pending && b.stream != stream) {
                const hipError_t q = hipEventQuery(b.done);
                if (q == hipErrorNotReady) {
                    if (other == v.size() || b.bytes < v[other].bytes) other = i;
                    continue;
                }
                if (q != hipSuccess) return map_err(q);
                b.pending = false;
            }
            if (best == v.size() || b.bytes < v[best].bytes) best = i;
        }
        const size_t live = (size_t)std::count_if(v.begin(), v.end(), [](const auto& b) { return b.p != nullptr; });
        if (best == v.size() && live >= kScratchMaxBlocks && other != v.size()) {
            CY_TRY(hipStreamWaitEvent(stream, v[other].done, 0));
            best = other;
        }
        if (best == v.size()) {
            uint64_t cap = 4096;
            while (cap < bytes) cap *= 2;
            trim(c, cap, victims);
            c->scratch_bytes += cap;
            *cap_out = cap;
            return CYAES_OK;
        }
        v[best].in_use = true;
        p = v[best].p;
        ctx = c;
        idx = best;
        s = stream;
        return CYAES_OK;
    }
    // Before caching `adding` more bytes: frees completed blocks, largest
    // first, while the cache would exceed kScratchCacheBytes (a large call's
    // block is not kept for the context's life).  Runs only when a
    // block is about to be allocated anyway and the cache is over its cap; the
    // blocks go to `victims`, freed by the caller after the mutex is released.
    static void trim(cyaes_gpu* c, uint64_t adding, std::vector<ScratchVictim>* victims) {
        auto& v = c->scratch;
        while (c->scratch_bytes + adding > kScratchCacheBytes) {
            size_t big = v.size();
            for (size_t i = 0; i < v.size(); i++) {
                const auto& b = v[i];
                if (!b.p || b.in_use || (b.pending && hipEventQuery(b.done) != hipSuccess)) continue;
                if (big == v.size() || b.bytes > v[big].bytes) big = i;
            }
            (void)hipGetLastError();
            if (big == v.size()) return;
            victims->push_back({v[big].p, v[big].done});
            c->scratch_bytes -= v[big].bytes;
            v[big] = {};  // an empty slot: the indices held by calls in flight stay valid
        }
    }
    ~StreamScratch() {
        if (!p) return;
        std::lock_guard<std::mutex> lk(ctx->scratch_mu);
        auto& b = ctx->scratch[idx];
        // after the kernels queued on s; if the record fails, the block stays
        // out of use until the context is destroyed (its synchronisation)
        b.pending = hipEventRecord(b.done, s) == hipSuccess;
        b.stream = s;
        b.in_use = !b.pending;
    }
};

// The whole 1,024-payload groups [0, nrag) of a ragged batch (unkeyed, no IV
// arrays; the plan of the lane kernel in `a`): k_encrypt_rag_lines walks by
// lines every wave whose payloads share a line phase and a length and hands
// the others back through a device list, which the lane kernel then walks.
int encrypt_rag_lines(cyaes_gpu* ctx, const EncArgs& a, uint64_t nrag, hipStream_t stream) {
    StreamScratch rest;
    int st = rest.get(ctx, 4 * (1 + nrag / 64), stream);
    if (st) return st;
    CY_TRY(hipMemsetAsync(rest.p, 0, 4, stream));
    EncArgs la = a;
    la.npayloads = nrag;
    la.rest = static_cast<uint32_t*>(rest.p);
    const Shape sh = wave_shape(ctx, nrag / 64, kEncThreads);
    const int grid = std::min(sh.grid, enc_grid_cap(ctx));
    CY_TRY(launch_encrypt_rag_lines(la, grid, sh.threads, stream));
    CY_TRY(launch_encrypt(la, grid, sh.threads, stream));  // the waves handed back (none for a relay stream)
    return note_key_use(ctx, la.keys.table, stream);
}

// d_iv_in == d_iv_out on a block-parallel decrypt: a payload's last block may
// be written before its first block reads the IV, so read from a copy.
int alias_iv(cyaes_gpu* ctx, StreamScratch& sc, const uint8_t** iv_in, const uint8_t* iv_out, uint64_t npayloads,
             hipStream_t stream) {
    if (!*iv_in || *iv_in != iv_out) return CYAES_OK;
    int st = sc.get(ctx, npayloads * 16, stream);
    if (st) return st;
    CY_TRY(hipMemcpyAsync(sc.p, *iv_in, npayloads * 16, hipMemcpyDeviceToDevice, stream));
    *iv_in = static_cast<const uint8_t*>(sc.p);
    return CYAES_OK;
}

// Uniform batch (off0 = stride = 0: contiguous), or a strided one (payload p at
// byte off0 + p * stride; unkeyed, no IV arrays, >= 64 blocks per payload, 32-bit
// payload indices and stride: the callers check).
// A flat decrypt's arguments, launch grid and per-launch scratch; the scratch
// blocks are released (behind the launch's kernels) when the plan goes out of
// scope.  dyn_pct: -1 the context's choice (long launches only), else the
// dynamic pool on with that share of the work (the duplex launch).
struct DecPlan {
    DecArgs a;
    int grid;
    StreamScratch iv_copy, boundary, work;
};

int dec_plan(cyaes_gpu* ctx, const uint8_t* in, uint8_t* out, uint64_t npayloads, uint32_t payload_bytes,
             const uint32_t* key_idx, uint32_t ppk, const uint8_t* iv_in, uint8_t* iv_out, hipStream_t stream,
             const uint32_t* table, uint32_t table_keys, uint64_t off0, uint64_t stride, int dyn_pct, int grid_want,
             DecPlan* plan) {
    DecArgs& a = plan->a;
    a = DecArgs{};
    a.off0 = off0;
    a.stride = stride;
    {
        const int ks = make_keysel(ctx, npayloads, key_idx, ppk, &a.keys, table, table_keys);
        if (ks) return ks;
    }
    if ((iv_in || iv_out) && npayloads > 0xFFFFFFFFull) return CYAES_EINVAL;
    const uint32_t bpp = payload_bytes / 16;
    const uint64_t nblocks = npayloads * bpp;
    const uint64_t step = 64ull * kDecRows;
    const uint64_t waves_needed = (nblocks + step - 1) / step;
    constexpr int kWaves = kDecThreads / 64;
    int grid = (int)std::min<uint64_t>((waves_needed + kWaves - 1) / kWaves, (uint64_t)dec_grid_cap(ctx));
    if (grid_want > 0) grid = grid_want;  // (the duplex grid: the encrypt's)
    plan->grid = grid;
    const uint64_t nwaves = (uint64_t)grid * kWaves;
    uint64_t bpw = (nblocks + nwaves - 1) / nwaves;  // the static split: one range per wave
    bpw = (bpw + step - 1) / step * step;
    StreamScratch &iv_copy = plan->iv_copy, &boundary = plan->boundary, &work = plan->work;
    int st = alias_iv(ctx, iv_copy, &iv_in, iv_out, npayloads, stream);
    if (st) return st;
    a.in = in;
    a.out = out;
    a.npayloads = npayloads;
    a.nblocks = nblocks;
    // Sessions of payloads_per_key payloads that are whole steps long: every
    // step lies in one session (the kernel picks its schedule per range).  Only
    // without IV arrays (the SESS kernels compile the IV code out).
    const uint64_t sess_blocks = (uint64_t)ppk * bpp;
    if (!key_idx && ppk && sess_blocks % step == 0 && !iv_in && !iv_out) a.sess_blocks = sess_blocks;
    // Work ranges (DecArgs, cyaes_device.h dyn_ticket).  Static split: one
    // range of bpw blocks per wave.  Dynamic (dyn): each wave first takes a
    // static range of (100 - dec_dyn_pct) % of its fair share, and the rest of
    // the batch is a pool of dec_range_steps-step ranges handed out by per-XCD
    // ticket pools with stealing, so waves on faster CUs and XCDs take more of
    // it and the waves finish within about one range of each other (the static
    // split's tail: CU and XCD speed spread, profiles/r04/timeline_*).  Per-lane
    // keys, IV arrays and sessions keep the static split (sessions: ranges that
    // divide the session).
    const bool keyed_lane = (key_idx || ppk) && !a.sess_blocks;
    const uint64_t fair_steps = bpw / step;
    const uint64_t dyn_steps = ctx->dec_range_steps;
    // Auto: only long launches (> kDecShortSteps steps per wave, config C) take the
    // pool; short ones level their waves by progress feedback alone (r04 A/B:
    // the pool cost config B 2-3 % and gained config C ~1 %).
    const bool dyn_want = dyn_pct >= 0 || ctx->dec_dyn == 1 || (ctx->dec_dyn < 0 && fair_steps > kDecShortSteps);
    a.dyn = dyn_want && !keyed_lane && !a.sess_blocks && !iv_in && !iv_out && dyn_steps > 0 &&
            dyn_steps < fair_steps;
    if (a.dyn) {
        const uint32_t pct = dyn_pct >= 0 ? (uint32_t)dyn_pct : ctx->dec_dyn_pct;
        uint64_t stat_steps = fair_steps * (100 - std::min<uint32_t>(pct, 100)) / 100;
        while (stat_steps && nwaves * stat_steps * step > nblocks) stat_steps--;
        a.stat_blocks = stat_steps * step;
        a.nstat = stat_steps ? (uint32_t)nwaves : 0;
        a.range_blocks = dyn_steps * step;
        const uint64_t ndyn = (nblocks - a.nstat * a.stat_blocks + a.range_blocks - 1) / a.range_blocks;
        a.nranges = a.nstat + ndyn;
        a.per_xcd = (uint32_t)((ndyn + kXcds - 1) / kXcds);
    } else {
        uint64_t range_steps = fair_steps;
        if (a.sess_blocks) {
            const uint64_t sess_steps = a.sess_blocks / step;
            while (sess_steps % range_steps) range_steps--;
        }
        a.stat_blocks = a.range_blocks = range_steps * step;
        a.nranges = (nblocks + a.stat_blocks - 1) / a.stat_blocks;
        a.nstat = (uint32_t)std::min<uint64_t>(a.nranges, 0xFFFFFFFFull);
    }
    if (a.nranges > 0xFFFFFFFFull) return CYAES_EINVAL;  // 32-bit tickets (> 2^40 blocks)
    // (A/B) XCD-weighted static split: out of place, static, one key, one range
    // per wave, whole workgroups per slot
    float wsum = 0.0f;
    for (uint32_t x = 0; x < kXcds; x++) wsum += ctx->dec_xcd_w[x];
    if (wsum > 0.0f && !a.dyn && in != out && !keyed_lane && !a.sess_blocks && !iv_in && !iv_out && grid_want <= 0 &&
        grid % (int)kXcds == 0 && stride == 0) {
        const uint64_t total = (nblocks + step - 1) / step, wpx = nwaves / kXcds;
        for (uint32_t x = 0; x < kXcds; x++)
            a.xsteps[x] = (uint32_t)std::ceil((double)total * ctx->dec_xcd_w[x] / wsum / (double)wpx);
        a.xw = 1;
        a.nstat = (uint32_t)nwaves;
        a.nranges = nwaves;
    }
    a.prio_short = fair_steps <= kDecShortSteps;
    a.bpp = make_fastdiv(bpp);
    a.step_q = (uint32_t)(step / bpp);
    a.step_r = (uint32_t)(step % bpp);
    a.iv_in = iv_in;
    a.iv_out = iv_out;
    a.tables = ctx->d_tables + kDecTableOff / 4;
    a.status = ctx->d_status;
    a.inplace = in == out;
    const uint32_t ww = dec_work_words((uint32_t)grid);
    st = work.get(ctx, 4ull * ww, stream);
    if (st) return st;
    a.work = static_cast<uint32_t*>(work.p);
    if (in == out && a.nranges > 1) {
        // A 32-B record per range.  Static ranges hand their carries over in the
        // kernel (records tagged with this launch's epoch: dec_handoff); dynamic
        // ones, whose ticket counters need the prepass anyway, have it snapshot them.
        const bool handoff = !a.dyn && ctx->dec_handoff;
        st = boundary.get(ctx, a.nranges * 2 * sizeof(uint4), stream);
        if (st) return st;
        a.boundary = static_cast<uint4*>(boundary.p);
        if (handoff) {
            static std::atomic<uint64_t> epochs{0};
            a.handoff = ++epochs;  // unique in the process: a recycled scratch block's old records never match
        }
    }
    // The ticket counter (dyn) and the boundary snapshot need the prepass; the
    // progress words are reset by their workgroups.  A small static batch (the
    // drop-in's packet) launches the kernel alone, as before.
    if (a.dyn || (a.boundary && !a.handoff)) CY_TRY(launch_dec_prepass(a, ww, stream));
    return CYAES_OK;
}

int decrypt_uniform(cyaes_gpu* ctx, const uint8_t* in, uint8_t* out, uint64_t npayloads, uint32_t payload_bytes,
                    const uint32_t* key_idx, uint32_t ppk, const uint8_t* iv_in, uint8_t* iv_out, hipStream_t stream,
                    const uint32_t* table = nullptr, uint32_t table_keys = 0, uint64_t off0 = 0, uint64_t stride = 0) {
    DecPlan plan;
    int st = dec_plan(ctx, in, out, npayloads, payload_bytes, key_idx, ppk, iv_in, iv_out, stream, table, table_keys,
                      off0, stride, -1, 0, &plan);
    if (st) return st;
    CY_TRY(launch_decrypt_flat(plan.a, plan.grid, stream));
    return note_key_use(ctx, plan.a.keys.table, stream);
}

int decrypt_ragged(cyaes_gpu* ctx, const uint8_t* in, uint8_t* out, const uint64_t* offsets, const uint32_t* nbytes,
                   uint64_t npayloads, const uint32_t* key_idx, uint32_t ppk, const uint8_t* iv_in, uint8_t* iv_out,
                   hipStream_t stream, const uint32_t* table = nullptr, uint32_t table_keys = 0, int max_grid = 0) {
    DecArgs a = {};
    int st = make_keysel(ctx, npayloads, key_idx, ppk, &a.keys, table, table_keys);
    if (st) return st;
    StreamScratch iv_copy;
    st = alias_iv(ctx, iv_copy, &iv_in, iv_out, npayloads, stream);
    if (st) return st;
    a.in = in;
    a.out = out;
    a.offsets = offsets;
    a.nbytes = nbytes;
    a.npayloads = npayloads;
    a.iv_in = iv_in;
    a.iv_out = iv_out;
    a.tables = ctx->d_tables + kDecTableOff / 4;
    a.status = ctx->d_status;
    a.inplace = in == out;
    // Payloads per wave group: as many as keep >= dec_groups_per_wave groups per
    // wave of a full grid (balance: with dynamic groups a wave takes the next
    // group from the launch's ticket counter, so the finer the groups the closer
    // the waves finish; static: >= 2), up to 64 (one holder lane each); small
    // payloads then share rows.  Sweeps in profiles/r01/ab_ragged_groups.txt, r04.
    // Dynamic groups by default when the batch has too few payloads for
    // 64-payload groups under the static split (fewer than 128 per wave of a
    // full grid): its payloads are then long, and their lengths uneven (a
    // relay stream of 0xFF00-B chunks and short tails: decrypt -25 % against
    // the static split, profiles/r06/ab/mixed_env.txt); many short payloads
    // (MTU packets) keep the static split (r04: the pool no faster there).
    const uint64_t slots = (uint64_t)std::max(1, ctx->num_cus) * (kDecThreads / 64);
    const bool dyn = ctx->dec_dyn == 1 || (ctx->dec_dyn < 0 && npayloads < 64 * 2 * slots);
    const uint64_t per_wave = dyn ? std::max<uint32_t>(1, ctx->dec_groups_per_wave) : 2;
    const uint64_t G = ctx->ragged_group ? ctx->ragged_group
                                         : std::min<uint64_t>(64, std::max<uint64_t>(1, npayloads / (per_wave * slots)));
    a.group = (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(1, G));
    a.nranges = (npayloads + a.group - 1) / a.group;
    if (a.nranges > 0xFFFFFFFFull) return CYAES_EINVAL;  // 32-bit tickets
    const Shape sh = wave_shape(ctx, a.nranges, kDecThreads);
    const int grid = std::min(std::min(sh.grid, dec_grid_cap(ctx)), max_grid > 0 ? max_grid : INT32_MAX);
    // Groups [0, nstat) static (strided over the waves), the rest a dynamic pool
    // from per-XCD ticket pools with stealing (as the flat kernel's ranges).
    const uint64_t nwaves = (uint64_t)grid * (sh.threads / 64);
    a.dyn = dyn && a.nranges > nwaves;
    if (a.dyn) {
        const uint64_t stat_per_wave = a.nranges * (100 - std::min<uint32_t>(ctx->dec_dyn_pct, 100)) / 100 / nwaves;
        a.nstat = (uint32_t)(stat_per_wave * nwaves);
        a.per_xcd = (uint32_t)((a.nranges - a.nstat + kXcds - 1) / kXcds);
    }
    StreamScratch work;
    const uint32_t ww = dec_work_words((uint32_t)grid);
    st = work.get(ctx, 4ull * ww, stream);
    if (st) return st;
    a.work = static_cast<uint32_t*>(work.p);
    if (a.dyn) CY_TRY(launch_dec_prepass(a, ww, stream));
    CY_TRY(launch_decrypt_ragged(a, grid, sh.threads, stream));
    return note_key_use(ctx, a.keys.table, stream);
}

bool aligned4(const void* p) { return ((uintptr_t)p & 3u) == 0; }

bool batch_args_ok(const cyaes_gpu* ctx, const uint8_t* in, const uint8_t* out, const void* iv_in,
                   const void* iv_out) {
    return ctx && in && out && aligned16(in) && aligned16(out) && aligned16(iv_in) && aligned16(iv_out);
}

// Ragged payloads may sit at any 4-byte-aligned offset (relay packets carry
// the payload at packet offset 12, relay_protocol.h:5-7,36-42).
bool ragged_args_ok(const cyaes_gpu* ctx, const uint8_t* in, const uint8_t* out, const void* iv_in,
                    const void* iv_out) {
    return ctx && in && out && aligned4(in) && aligned4(out) && aligned16(iv_in) && aligned16(iv_out);
}

}  // namespace

static void destroy_pipe(HostPipe* p);

int cyaes::ragged_batch(cyaes_gpu* ctx, bool decrypt, const uint32_t* d_table, uint32_t table_keys,
                        const uint8_t* in, uint8_t* out, const uint64_t* offsets, const uint32_t* nbytes,
                        uint64_t npayloads, const uint32_t* key_idx, hipStream_t stream) {
    if (!ctx || !d_table || !offsets || !nbytes || !ragged_args_ok(ctx, in, out, nullptr, nullptr)) return CYAES_EINVAL;
    if (npayloads == 0) return CYAES_OK;
    DeviceGuard g(ctx->device);
    return decrypt ? decrypt_ragged(ctx, in, out, offsets, nbytes, npayloads, key_idx, 0, nullptr, nullptr, stream,
                                    d_table, table_keys)
                   : encrypt_common(ctx, in, out, offsets, nbytes, npayloads, 0, key_idx, 0, nullptr, nullptr, stream,
                                    d_table, table_keys);
}

extern "C" {

const uint8_t* cyaes_default_iv(void) {
    static const uint8_t iv[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
    return iv;
}

const char* cyaes_strerror(int status) {
    switch (status) {
        case CYAES_OK: return "ok";
        case CYAES_EINVAL: return "invalid argument";
        case CYAES_EDEVICE: return "HIP device error";
        case CYAES_ENOMEM: return "out of memory";
        case CYAES_ERANGE: return "key index out of range";
        case CYAES_ENODEV: return "no gfx950 device";
        default: return "unknown status";
    }
}

const char* cyaes_version(void) { return "cyaes-mi355x 0.1.0 (gfx950, AES-128-CBC, cyclone::Rijndael drop-in)"; }

int cyaes_key_expand(const uint8_t key[16], cyaes_key* out) {
    if (!key || !out) return CYAES_EINVAL;
    expand_key(key, out);
    return CYAES_OK;
}

int cyaes_gpu_create(int device, cyaes_gpu** out) {
    if (!out) return CYAES_EINVAL;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return CYAES_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return CYAES_ENODEV;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return CYAES_ENODEV;
    DeviceGuard g(device);
    if (!g.ok) return CYAES_ENODEV;
    cyaes_gpu* ctx = new cyaes_gpu();
    ctx->device = device;
    ctx->num_cus = prop.multiProcessorCount;
    if (const char* q = getenv("CYAES_QUAD_MAX_CHAINS")) ctx->quad_max_chains = strtoull(q, nullptr, 10);
    if (const char* g = getenv("CYAES_RAGGED_GROUP")) ctx->ragged_group = (uint32_t)strtoul(g, nullptr, 10);
    if (const char* r = getenv("CYAES_ENC_RUN")) ctx->enc_run = (uint32_t)strtoul(r, nullptr, 10);
    if (const char* v = getenv("CYAES_ENC_NO_SESS")) ctx->enc_no_sess = atoi(v) != 0;
    if (const char* v = getenv("CYAES_ENC_LINES")) ctx->enc_no_lines = atoi(v) == 0;
    if (const char* v = getenv("CYAES_LINES_GRID")) ctx->lines_grid = atoi(v);
    if (const char* v = getenv("CYAES_ENC_RAG_LINES")) ctx->enc_no_rag_lines = atoi(v) == 0;
    if (const char* v = getenv("CYAES_DEC_DYN")) ctx->dec_dyn = atoi(v) != 0 ? 1 : 0;
    if (const char* v = getenv("CYAES_DEC_RANGE_STEPS")) ctx->dec_range_steps = (uint32_t)strtoul(v, nullptr, 10);
    if (const char* v = getenv("CYAES_DEC_GROUPS_PER_WAVE")) ctx->dec_groups_per_wave = (uint32_t)strtoul(v, nullptr, 10);
    if (const char* v = getenv("CYAES_DEC_GRID")) ctx->dec_grid_max = atoi(v);
    if (const char* v = getenv("CYAES_DEC_XCD_W")) {
        float w[kXcds];
        if (sscanf(v, "%f,%f,%f,%f,%f,%f,%f,%f", &w[0], &w[1], &w[2], &w[3], &w[4], &w[5], &w[6], &w[7]) == (int)kXcds)
            for (uint32_t x = 0; x < kXcds; x++) ctx->dec_xcd_w[x] = std::max(0.0f, w[x]);
    }
    if (const char* v = getenv("CYAES_DEC_DYN_PCT")) ctx->dec_dyn_pct = (uint32_t)strtoul(v, nullptr, 10);
    if (const char* v = getenv("CYAES_STRIDED_LISTS")) ctx->strided_lists = atoi(v) != 0;
    if (const char* v = getenv("CYAES_STRIDED_FORCE")) ctx->strided_force = atoi(v) != 0;
    if (const char* v = getenv("CYAES_DEC_HANDOFF")) ctx->dec_handoff = atoi(v) != 0;
    if (const char* v = getenv("CYAES_DUPLEX")) ctx->duplex_off = atoi(v) == 0;
    if (const char* v = getenv("CYAES_DUPLEX_PACK")) ctx->duplex_pack = std::max(1, std::min(16, atoi(v)));
    if (const char* v = getenv("CYAES_DUPLEX_DEC_WGS")) ctx->dup_min_dec_wgs = std::max(1, atoi(v));
    if (const char* v = getenv("CYAES_DUPLEX_DYN_PCT")) ctx->duplex_dyn_pct = (uint32_t)strtoul(v, nullptr, 10);
    const HostTables& t = host_tables();
    uint8_t host[kTablesBytes];
    memcpy(host + kEncTableOff, t.enc, sizeof(t.enc));
    memcpy(host + kDecTableOff, t.dec, sizeof(t.dec));
    memcpy(host + kSboxOff, t.sbox, 256);
    memcpy(host + kSiOff, t.inv_sbox, 256);
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&ctx->d_tables), kTablesBytes);
    if (e == hipSuccess) e = hipMemcpy(ctx->d_tables, host, kTablesBytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&ctx->d_status), 16);
    if (e == hipSuccess) e = hipMemset(ctx->d_status, 0, 16);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&ctx->d_digest), 16);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->keys_written, hipEventDisableTiming);
    if (e != hipSuccess) {
        cyaes_gpu_destroy(ctx);
        return map_err(e);
    }
    *out = ctx;
    return CYAES_OK;
}

int cyaes_gpu_destroy(cyaes_gpu* ctx) {
    if (!ctx) return CYAES_OK;
    DeviceGuard g(ctx->device);
    // The device-wide synchronisation reports any fault still pending from this
    // context's work (or anything else on the device): the caller learns of it
    // here, not from the next context's first call.
    const hipError_t e = hipDeviceSynchronize();
    (void)hipFree(ctx->d_tables);
    (void)hipFree(ctx->d_keys);
    (void)hipFree(ctx->d_status);
    (void)hipFree(ctx->d_digest);
    for (uint32_t* k : ctx->retired_keys) (void)hipFree(k);
    destroy_pipe(ctx->pipe);
    for (auto& b : ctx->scratch) {  // (every batch has completed: the synchronisation above)
        if (!b.p) continue;
        (void)hipFree(b.p);
        (void)hipEventDestroy(b.done);
    }
    for (auto& u : ctx->key_uses) (void)hipEventDestroy(u.second);
    if (ctx->keys_written) (void)hipEventDestroy(ctx->keys_written);
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    delete ctx;
    return map_err(e);
}

int cyaes_gpu_device(const cyaes_gpu* ctx) { return ctx ? ctx->device : -1; }
int cyaes_gpu_num_cus(const cyaes_gpu* ctx) { return ctx ? ctx->num_cus : 0; }
uint32_t cyaes_gpu_nkeys(const cyaes_gpu* ctx) { return ctx ? ctx->nkeys : 0; }

int cyaes_debug_ctx(cyaes_gpu* ctx, uint64_t out[4]) {
    if (!ctx || !out) return CYAES_EINVAL;
    {
        std::lock_guard<std::mutex> lk(ctx->key_mu);
        out[0] = ctx->key_uses.size();
        out[3] = ctx->retired_keys.size();
    }
    std::lock_guard<std::mutex> lk(ctx->scratch_mu);
    out[1] = (uint64_t)std::count_if(ctx->scratch.begin(), ctx->scratch.end(), [](const auto& b) { return b.p != nullptr; });
    out[2] = ctx->scratch_bytes;
    return CYAES_OK;
}

// A private non-blocking stream for one key-table copy, destroyed after it.
// Not kept in the context: the box gives a process 4 hardware queues
// (GPU_MAX_HW_QUEUES) and streams beyond that share them, so a context-lifetime
// stream here made the host pipe's upload and compute streams share a queue
// (e2e encrypt 42.8 -> 31.9 GiB/s, back to 43.5 with 8 queues;
// profiles/r05/e2e_hw_queues.txt).
struct KeyStream {
    hipStream_t s = nullptr;
    hipError_t e;
    KeyStream() { e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking); }
    ~KeyStream() {
        if (s) (void)hipStreamDestroy(s);
    }
};

// The key table's writers wait only for the streams that read it: each
// stream's last batch under this context's table (note_key_use), and an
// expansion cyaes_gpu_set_keys_device queued on a caller's stream.
static int wait_key_readers(cyaes_gpu* ctx) {
    std::lock_guard<std::mutex> lk(ctx->key_mu);
    for (auto& u : ctx->key_uses) CY_TRY(hipEventSynchronize(u.second));
    for (auto& u : ctx->key_uses) (void)hipEventDestroy(u.second);  // all complete: nothing left to wait for
    ctx->key_uses.clear();
    return CYAES_OK;
}
static int wait_key_writes(cyaes_gpu* ctx) {
    if (ctx->keys_written_pending) {
        CY_TRY(hipEventSynchronize(ctx->keys_written));
        ctx->keys_written_pending = false;
    }
    return CYAES_OK;
}

// Grows the table to hold nkeys rows.  The outgrown table is kept until the
// context is destroyed (batches queued before may still read it; hipFree
// would wait for the whole device), so a grown table needs no wait at all.
// *grown tells whether the table is new (nothing reads it yet).
static int reserve_keys(cyaes_gpu* ctx, uint32_t nkeys, uint32_t keep_rows, bool* grown) {
    *grown = false;
    if (ctx->key_cap >= nkeys) return CYAES_OK;
    const uint32_t cap = std::max(nkeys, ctx->key_cap * 2);
    uint32_t* t = nullptr;
    CY_TRY(hipMalloc(reinterpret_cast<void**>(&t), (uint64_t)cap * kSchedWords * 4));
    if (keep_rows) {
        int st = wait_key_writes(ctx);
        KeyStream ks;
        hipError_t e = st ? hipErrorUnknown : ks.e;
        if (e == hipSuccess)
            e = hipMemcpyAsync(t, ctx->d_keys, (uint64_t)keep_rows * kSchedWords * 4, hipMemcpyDeviceToDevice, ks.s);
        if (e == hipSuccess) e = hipStreamSynchronize(ks.s);
        if (e != hipSuccess) {
            (void)hipFree(t);
            return st ? st : map_err(e);
        }
    }
    if (ctx->d_keys) ctx->retired_keys.push_back(ctx->d_keys);
    ctx->d_keys = t;
    ctx->key_cap = cap;
    *grown = true;
    return CYAES_OK;
}

// Writes rows [first, first + n) from host schedules: in place only after the
// streams that read the table are done with it.
static int write_key_rows(cyaes_gpu* ctx, uint32_t first, const uint32_t* host, uint32_t n, bool fresh_table) {
    if (!fresh_table) {
        int st = wait_key_readers(ctx);
        if (st) return st;
    }
    int st = wait_key_writes(ctx);
    if (st) return st;
    KeyStream ks;
    CY_TRY(ks.e);
    CY_TRY(hipMemcpyAsync(ctx->d_keys + (uint64_t)first * kSchedWords, host, (uint64_t)n * kSchedWords * 4,
                          hipMemcpyHostToDevice, ks.s));
    CY_TRY(hipStreamSynchronize(ks.s));
    return CYAES_OK;
}

int cyaes_gpu_set_keys(cyaes_gpu* ctx, const uint8_t* keys, uint32_t nkeys) {
    if (!ctx || !keys || nkeys == 0) return CYAES_EINVAL;
    DeviceGuard g(ctx->device);
    std::vector<uint32_t> host((size_t)nkeys * kSchedWords);
    for (uint32_t i = 0; i < nkeys; i++) {
        cyaes_key k;
        expand_key(keys + 16ull * i, &k);
        to_device_schedule(k, host.data() + (size_t)i * kSchedWords);
    }
    bool grown = false;
    int st = reserve_keys(ctx, nkeys, 0, &grown);
    if (st) return st;
    st = write_key_rows(ctx, 0, host.data(), nkeys, grown);
    if (st) return st;
    ctx->nkeys = nkeys;
    return CYAES_OK;
}

int cyaes_gpu_update_keys(cyaes_gpu* ctx, uint32_t first, const uint8_t* keys, uint32_t n) {
    if (!ctx || !keys || n == 0 || first > ctx->nkeys || (uint64_t)first + n > 0xFFFFFFFFull) return CYAES_EINVAL;
    DeviceGuard g(ctx->device);
    const uint32_t total = std::max(ctx->nkeys, first + n);
    std::vector<uint32_t> host((size_t)n * kSchedWords);
    for (uint32_t i = 0; i < n; i++) {
        cyaes_key k;
        expand_key(keys + 16ull * i, &k);
        to_device_schedule(k, host.data() + (size_t)i * kSchedWords);
    }
    bool grown = false;  // grow, keeping rows [0, first)
    int st = reserve_keys(ctx, total, first, &grown);
    if (st) return st;
    // Appended rows only (first == nkeys) are rows no queued batch can read either.
    st = write_key_rows(ctx, first, host.data(), n, grown || first == ctx->nkeys);
    if (st) return st;
    ctx->nkeys = total;
    return CYAES_OK;
}

int cyaes_gpu_set_keys_device(cyaes_gpu* ctx, const uint8_t* d_keys, uint32_t nkeys, void* stream) {
    if (!ctx || !d_keys || nkeys == 0) return CYAES_EINVAL;
    DeviceGuard g(ctx->device);
    bool grown = false;
    int st = reserve_keys(ctx, nkeys, 0, &grown);
    if (st) return st;
    hipStream_t s = (hipStream_t)stream;
    if (!grown) {  // the expansion waits (on the device) for the streams still reading the table
        std::lock_guard<std::mutex> lk(ctx->key_mu);
        for (auto& u : ctx->key_uses)
            if (u.first != s) CY_TRY(hipStreamWaitEvent(s, u.second, 0));
    }
    // ... and for an expansion still pending from an earlier set_keys_device
    // on another stream (r06): rows are written in call
    // order, and keys_written, re-recorded below, then covers both.
    if (ctx->keys_written_pending) CY_TRY(hipStreamWaitEvent(s, ctx->keys_written, 0));
    const uint8_t* d_sbox = reinterpret_cast<const uint8_t*>(ctx->d_tables) + kSboxOff;
    CY_TRY(launch_key_expand(d_keys, nkeys, d_sbox, ctx->d_keys, s));
    CY_TRY(hipEventRecord(ctx->keys_written, s));
    ctx->keys_written_pending = true;
    ctx->nkeys = nkeys;
    return CYAES_OK;
}

int cyaes_gpu_get_key(cyaes_gpu* ctx, uint32_t index, cyaes_key* out) {
    if (!ctx || !out) return CYAES_EINVAL;
    if (index >= ctx->nkeys) return CYAES_ERANGE;
    DeviceGuard g(ctx->device);
    uint32_t w[kSchedWords];
    int st = wait_key_writes(ctx);
    if (st) return st;
    KeyStream ks;
    CY_TRY(ks.e);
    CY_TRY(hipMemcpyAsync(w, ctx->d_keys + (uint64_t)index * kSchedWords, sizeof(w), hipMemcpyDeviceToHost, ks.s));
    CY_TRY(hipStreamSynchronize(ks.s));
    from_device_schedule(w, out);
    return CYAES_OK;
}

// Zero-length chains: the final chain is the initial chain (the reference's
// loop never runs and writes the IV back unchanged, cyr_rijndael.cpp:600-608).
static int empty_chains(cyaes_gpu* ctx, uint64_t npayloads, const uint32_t* key_idx, uint32_t ppk,
                        const uint8_t* iv_in, uint8_t* iv_out, void* stream) {
    if (!iv_out) return CYAES_OK;
    if (!aligned16(iv_in) || !aligned16(iv_out)) return CYAES_EINVAL;
    static uint8_t dummy_storage[16] __attribute__((aligned(16)));  // never dereferenced: no blocks
    DeviceGuard g(ctx->device);
    return encrypt_common(ctx, dummy_storage, dummy_storage, nullptr, nullptr, npayloads, 0, key_idx, ppk, iv_in,
                          iv_out, (hipStream_t)stream);
}

int cyaes_gpu_encrypt_uniform(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, uint64_t npayloads,
                              uint32_t payload_bytes, const uint32_t* d_key_idx, uint32_t payloads_per_key,
                              const uint8_t* d_iv_in, uint8_t* d_iv_out, void* stream) {
    if (!ctx || payload_bytes % 16) return CYAES_EINVAL;
    if (npayloads == 0) return CYAES_OK;
    if (payload_bytes == 0) return empty_chains(ctx, npayloads, d_key_idx, payloads_per_key, d_iv_in, d_iv_out, stream);
    if (!batch_args_ok(ctx, d_in, d_out, d_iv_in, d_iv_out)) return CYAES_EINVAL;
    DeviceGuard g(ctx->device);
    return encrypt_common(ctx, d_in, d_out, nullptr, nullptr, npayloads, payload_bytes, d_key_idx, payloads_per_key,
                          d_iv_in, d_iv_out, (hipStream_t)stream);
}

int cyaes_gpu_decrypt_uniform(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, uint64_t npayloads,
                              uint32_t payload_bytes, const uint32_t* d_key_idx, uint32_t payloads_per_key,
                              const uint8_t* d_iv_in, uint8_t* d_iv_out, void* stream) {
    if (!ctx || payload_bytes % 16) return CYAES_EINVAL;
    if (npayloads == 0) return CYAES_OK;
    if (payload_bytes == 0) return empty_chains(ctx, npayloads, d_key_idx, payloads_per_key, d_iv_in, d_iv_out, stream);
    if (!batch_args_ok(ctx, d_in, d_out, d_iv_in, d_iv_out)) return CYAES_EINVAL;
    DeviceGuard g(ctx->device);
    return decrypt_uniform(ctx, d_in, d_out, npayloads, payload_bytes, d_key_idx, payloads_per_key, d_iv_in, d_iv_out,
                           (hipStream_t)stream);
}

int cyaes_gpu_encrypt_ragged(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, const uint64_t* d_offsets,
                             const uint32_t* d_nbytes, uint64_t npayloads, const uint32_t* d_key_idx,
                             uint32_t payloads_per_key, const uint8_t* d_iv_in, uint8_t* d_iv_out, void* stream) {
    if (!ctx) return CYAES_EINVAL;
    if (npayloads == 0) return CYAES_OK;
    if (!d_offsets || !d_nbytes || !ragged_args_ok(ctx, d_in, d_out, d_iv_in, d_iv_out)) return CYAES_EINVAL;
    DeviceGuard g(ctx->device);
    return encrypt_common(ctx, d_in, d_out, d_offsets, d_nbytes, npayloads, 0, d_key_idx, payloads_per_key, d_iv_in,
                          d_iv_out, (hipStream_t)stream);
}

int cyaes_gpu_decrypt_ragged(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, const uint64_t* d_offsets,
                             const uint32_t* d_nbytes, uint64_t npayloads, const uint32_t* d_key_idx,
                             uint32_t payloads_per_key, const uint8_t* d_iv_in, uint8_t* d_iv_out, void* stream) {
    if (!ctx) return CYAES_EINVAL;
    if (npayloads == 0) return CYAES_OK;
    if (!d_offsets || !d_nbytes || !ragged_args_ok(ctx, d_in, d_out, d_iv_in, d_iv_out)) return CYAES_EINVAL;
    DeviceGuard g(ctx->device);
    return decrypt_ragged(ctx, d_in, d_out, d_offsets, d_nbytes, npayloads, d_key_idx, payloads_per_key, d_iv_in,
                          d_iv_out, (hipStream_t)stream);
}

int cyaes_gpu_cbc_encrypt_batch(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, const uint64_t* d_offsets,
                                const uint32_t* d_nbytes, const uint32_t* d_key_idx, const uint8_t* d_iv,
                                uint32_t npayloads, void* stream) {
    return cyaes_gpu_encrypt_ragged(ctx, d_in, d_out, d_offsets, d_nbytes, npayloads, d_key_idx, 0, d_iv, nullptr,
                                    stream);
}

int cyaes_gpu_cbc_decrypt_batch(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, const uint64_t* d_offsets,
                                const uint32_t* d_nbytes, const uint32_t* d_key_idx, const uint8_t* d_iv,
                                uint32_t npayloads, void* stream) {
    return cyaes_gpu_decrypt_ragged(ctx, d_in, d_out, d_offsets, d_nbytes, npayloads, d_key_idx, 0, d_iv, nullptr,
                                    stream);
}

// Strided batches: the encrypt runs the ragged kernels with positions computed
// from the stride; the decrypt runs the flat kernel's STRIDED addressing when
// it applies (unkeyed, >= 64 blocks per payload: the relay's MTU packets), and
// otherwise the ragged kernel with the two lists written on the device first
// (12 B per payload; CYAES_STRIDED_LISTS=1 forces that for both, tests / A/B).
static int strided_batch(cyaes_gpu* ctx, bool decrypt, const uint8_t* in, uint8_t* out, uint64_t first,
                         uint64_t stride, uint64_t npayloads, uint32_t payload_bytes, const uint32_t* key_idx,
                         uint32_t ppk, hipStream_t stream) {
    if (!ctx || payload_bytes % 16 || first % 4 || stride % 4 || stride < payload_bytes) return CYAES_EINVAL;
    if (npayloads == 0 || payload_bytes == 0) return CYAES_OK;
    if (!ragged_args_ok(ctx, in, out, nullptr, nullptr)) return CYAES_EINVAL;
    if (npayloads - 1 > (UINT64_MAX - first - payload_bytes) / stride) return CYAES_EINVAL;
    DeviceGuard g(ctx->device);
    const uint32_t bpp = payload_bytes / 16;
    // Back-to-back payloads, 16-B aligned: a contiguous uniform batch
    if (stride == payload_bytes && !ctx->strided_force && batch_args_ok(ctx, in + first, out + first, nullptr, nullptr))
        return decrypt ? decrypt_uniform(ctx, in + first, out + first, npayloads, payload_bytes, key_idx, ppk, nullptr,
                                         nullptr, stream)
                       : encrypt_common(ctx, in + first, out + first, nullptr, nullptr, npayloads, payload_bytes,
                                        key_idx, ppk, nullptr, nullptr, stream);
    // The flat kernel's strided rows use 32-bit byte offsets from the stream's first payload
    const bool span32 = (npayloads - 1) * stride + payload_bytes <= 0xFFFFFFFFull;
    if (decrypt && !key_idx && !ppk && bpp >= 64 && span32 && !ctx->strided_lists)
        return decrypt_uniform(ctx, in, out, npayloads, payload_bytes, nullptr, 0, nullptr, nullptr, stream, nullptr, 0,
                               first, stride);
    if (!decrypt && !ctx->strided_lists)  // the ragged encrypt kernels compute the positions themselves
        return encrypt_common(ctx, in, out, nullptr, nullptr, npayloads, payload_bytes, key_idx, ppk, nullptr, nullptr,
                              stream, nullptr, 0, first, stride);
    StreamScratch lists;
    int st = lists.get(ctx, npayloads * 12, stream);
    if (st) return st;
    uint64_t* offs = static_cast<uint64_t*>(lists.p);
    uint32_t* nb = reinterpret_cast<uint32_t*>(offs + npayloads);
    CY_TRY(launch_strided_lists(offs, nb, first, stride, npayloads, payload_bytes, stream));
    return decrypt ? decrypt_ragged(ctx, in, out, offs, nb, npayloads, key_idx, ppk, nullptr, nullptr, stream)
                   : encrypt_common(ctx, in, out, offs, nb, npayloads, 0, key_idx, ppk, nullptr, nullptr, stream);
}

int cyaes_gpu_encrypt_strided(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, uint64_t first_offset,
                              uint64_t stride, uint64_t npayloads, uint32_t payload_bytes, const uint32_t* d_key_idx,
                              uint32_t payloads_per_key, void* stream) {
    return strided_batch(ctx, false, d_in, d_out, first_offset, stride, npayloads, payload_bytes, d_key_idx,
                         payloads_per_key, (hipStream_t)stream);
}

int cyaes_gpu_decrypt_strided(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, uint64_t first_offset,
                              uint64_t stride, uint64_t npayloads, uint32_t payload_bytes, const uint32_t* d_key_idx,
                              uint32_t payloads_per_key, void* stream) {
    return strided_batch(ctx, true, d_in, d_out, first_offset, stride, npayloads, payload_bytes, d_key_idx,
                         payloads_per_key, (hipStream_t)stream);
}

// Duplex: one batch encrypted and another decrypted in one launch
// (cyaes_duplex_kernels.hip).  Falls back to the two ordinary launches, in
// that order, whenever the duplex grid does not apply: a half too small to
// fill the GPU on its own (the quad encrypt, or a decrypt without a dynamic
// pool), or batches whose bytes overlap (the two halves run concurrently).
static bool overlaps(const uint8_t* a, uint64_t na, const uint8_t* b, uint64_t nb) {
    return (uintptr_t)a < (uintptr_t)b + nb && (uintptr_t)b < (uintptr_t)a + na;
}

int cyaes_gpu_duplex_uniform(cyaes_gpu* ctx, const uint8_t* d_enc_in, uint8_t* d_enc_out, uint64_t enc_npayloads,
                             uint32_t enc_payload_bytes, uint32_t enc_key, const uint8_t* d_dec_in, uint8_t* d_dec_out,
                             uint64_t dec_npayloads, uint32_t dec_payload_bytes, uint32_t dec_key, void* stream) {
    if (!ctx || enc_payload_bytes % 16 || dec_payload_bytes % 16) return CYAES_EINVAL;
    const bool has_e = enc_npayloads && enc_payload_bytes, has_d = dec_npayloads && dec_payload_bytes;
    if (has_e && !batch_args_ok(ctx, d_enc_in, d_enc_out, nullptr, nullptr)) return CYAES_EINVAL;
    if (has_d && !batch_args_ok(ctx, d_dec_in, d_dec_out, nullptr, nullptr)) return CYAES_EINVAL;
    if ((has_e && enc_key >= ctx->nkeys) || (has_d && dec_key >= ctx->nkeys)) return CYAES_ERANGE;
    if (!has_e && !has_d) return CYAES_OK;
    DeviceGuard g(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t* te = ctx->d_keys + (uint64_t)enc_key * kSchedWords;
    const uint32_t* td = ctx->d_keys + (uint64_t)dec_key * kSchedWords;
    auto sequential = [&]() -> int {
        if (has_e) {
            const int st = encrypt_common(ctx, d_enc_in, d_enc_out, nullptr, nullptr, enc_npayloads, enc_payload_bytes,
                                          nullptr, 0, nullptr, nullptr, s, te, 1);
            if (st) return st;
        }
        return has_d ? decrypt_uniform(ctx, d_dec_in, d_dec_out, dec_npayloads, dec_payload_bytes, nullptr, 0, nullptr,
                                       nullptr, s, td, 1)
                     : CYAES_OK;
    };
    if (!has_e || !has_d || ctx->duplex_off) return sequential();
    const uint64_t eb = enc_npayloads * enc_payload_bytes, db = dec_npayloads * dec_payload_bytes;
    if (overlaps(d_enc_out, eb, d_dec_in, db) || overlaps(d_enc_out, eb, d_dec_out, db) ||
        overlaps(d_dec_out, db, d_enc_in, eb))
        return sequential();
    EncPlan ep;
    int st = enc_plan(ctx, d_enc_in, d_enc_out, nullptr, nullptr, enc_npayloads, enc_payload_bytes, nullptr, 0, nullptr,
                      nullptr, te, 1, 0, 0, &ep);
    if (st) return st;
    if (ep.quad || ep.sess || ep.threads != kDecThreads) return sequential();
    DecPlan dp;
    st = dec_plan(ctx, d_dec_in, d_dec_out, dec_npayloads, dec_payload_bytes, nullptr, 0, nullptr, nullptr, s, td, 1, 0,
                  0, (int)ctx->duplex_dyn_pct, ep.grid, &dp);
    if (st) return st;
    if (!dp.a.dyn) {  // (its prepass, if any, only zeroed scratch words)
        CY_TRY(launch_encrypt(ep.a, ep.grid, ep.threads, s));
        CY_TRY(launch_decrypt_flat(dp.a, dp.grid, s));
        return note_key_use(ctx, te, s);
    }
    DuplexArgs x;
    x.e = ep.a;
    x.d = dp.a;
    CY_TRY(launch_duplex(x, ep.grid, s));
    return note_key_use(ctx, te, s);
}

// Duplex of two relay streams (r06): the sender's stream
// encrypted by 64-B lines while the receiver's is decrypted by the flat
// kernel's strided rows, in one grid.  Same results as
//   cyaes_gpu_encrypt_strided(enc stream, key row enc_key)
//   cyaes_gpu_decrypt_strided(dec stream, key row dec_key)
// in that order; whenever one half would not take those kernels (short or
// unaligned streams, spans past 32-bit offsets, overlapping streams) it runs
// as exactly those two calls.
int cyaes_gpu_duplex_strided(cyaes_gpu* ctx, const uint8_t* d_enc_in, uint8_t* d_enc_out, uint64_t enc_first,
                             uint64_t enc_stride, uint64_t enc_npayloads, uint32_t enc_payload_bytes, uint32_t enc_key,
                             const uint8_t* d_dec_in, uint8_t* d_dec_out, uint64_t dec_first, uint64_t dec_stride,
                             uint64_t dec_npayloads, uint32_t dec_payload_bytes, uint32_t dec_key, void* stream) {
    if (!ctx) return CYAES_EINVAL;
    const bool has_e = enc_npayloads && enc_payload_bytes, has_d = dec_npayloads && dec_payload_bytes;
    auto half_ok = [&](const uint8_t* in, const uint8_t* out, uint64_t first, uint64_t stride, uint64_t n,
                       uint32_t pb) {
        return pb % 16 == 0 && first % 4 == 0 && stride % 4 == 0 && stride >= pb && ragged_args_ok(ctx, in, out, nullptr, nullptr) &&
               n - 1 <= (UINT64_MAX - first - pb) / stride;
    };
    if (enc_payload_bytes % 16 || dec_payload_bytes % 16) return CYAES_EINVAL;
    if (has_e && !half_ok(d_enc_in, d_enc_out, enc_first, enc_stride, enc_npayloads, enc_payload_bytes))
        return CYAES_EINVAL;
    if (has_d && !half_ok(d_dec_in, d_dec_out, dec_first, dec_stride, dec_npayloads, dec_payload_bytes))
        return CYAES_EINVAL;
    if ((has_e && enc_key >= ctx->nkeys) || (has_d && dec_key >= ctx->nkeys)) return CYAES_ERANGE;
    if (!has_e && !has_d) return CYAES_OK;
    DeviceGuard g(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t* te = ctx->d_keys + (uint64_t)enc_key * kSchedWords;
    const uint32_t* td = ctx->d_keys + (uint64_t)dec_key * kSchedWords;
    const uint64_t espan = has_e ? (enc_npayloads - 1) * enc_stride + enc_payload_bytes : 0;
    const uint64_t dspan = has_d ? (dec_npayloads - 1) * dec_stride + dec_payload_bytes : 0;
    auto sequential = [&]() -> int {
        if (has_e) {  // (the strided entry points' own kernel choice, under the key row)
            const int st = enc_stride == enc_payload_bytes && batch_args_ok(ctx, d_enc_in + enc_first, d_enc_out + enc_first, nullptr, nullptr)
                               ? encrypt_common(ctx, d_enc_in + enc_first, d_enc_out + enc_first, nullptr, nullptr,
                                                enc_npayloads, enc_payload_bytes, nullptr, 0, nullptr, nullptr, s, te, 1)
                               : encrypt_common(ctx, d_enc_in, d_enc_out, nullptr, nullptr, enc_npayloads,
                                                enc_payload_bytes, nullptr, 0, nullptr, nullptr, s, te, 1, enc_first,
                                                enc_stride);
            if (st) return st;
        }
        if (!has_d) return CYAES_OK;
        if (dec_stride == dec_payload_bytes && batch_args_ok(ctx, d_dec_in + dec_first, d_dec_out + dec_first, nullptr, nullptr))
            return decrypt_uniform(ctx, d_dec_in + dec_first, d_dec_out + dec_first, dec_npayloads, dec_payload_bytes,
                                   nullptr, 0, nullptr, nullptr, s, td, 1);
        if (dec_payload_bytes / 16 >= 64 && dspan <= 0xFFFFFFFFull && !ctx->strided_lists)
            return decrypt_uniform(ctx, d_dec_in, d_dec_out, dec_npayloads, dec_payload_bytes, nullptr, 0, nullptr,
                                   nullptr, s, td, 1, dec_first, dec_stride);
        StreamScratch lists;
        int st = lists.get(ctx, dec_npayloads * 12, s);
        if (st) return st;
        uint64_t* offs = static_cast<uint64_t*>(lists.p);
        uint32_t* nb = reinterpret_cast<uint32_t*>(offs + dec_npayloads);
        CY_TRY(launch_strided_lists(offs, nb, dec_first, dec_stride, dec_npayloads, dec_payload_bytes, s));
        return decrypt_ragged(ctx, d_dec_in, d_dec_out, offs, nb, dec_npayloads, nullptr, 0, nullptr, nullptr, s, td, 1);
    };
    if (!has_e || !has_d || ctx->duplex_off) return sequential();
    // The duplex form: the encrypt half's whole line groups by lines, its
    // decrypt half by the flat strided rows; 16-B aligned back-to-back streams
    // are uniform batches (cyaes_gpu_duplex_uniform's business).
    const uint64_t nlines = enc_npayloads / kLinesGroup * kLinesGroup;
    const bool e_lines = !ctx->enc_no_lines && enc_stride != enc_payload_bytes && nlines &&
                         (nlines - 1) * enc_stride + enc_payload_bytes + enc_first + 64 <= 0xFFFFFFFFull &&
                         !ragged_encrypt_is_quad(ctx, enc_npayloads);
    const bool d_flat = dec_stride != dec_payload_bytes && dec_payload_bytes / 16 >= 64 && dspan <= 0xFFFFFFFFull &&
                        !ctx->strided_lists;
    if (!e_lines || !d_flat || overlaps(d_enc_out + enc_first, espan, d_dec_in + dec_first, dspan) ||
        overlaps(d_enc_out + enc_first, espan, d_dec_out + dec_first, dspan) ||
        overlaps(d_dec_out + dec_first, dspan, d_enc_in + enc_first, espan))
        return sequential();
    EncPlan ep;
    int st = enc_plan(ctx, d_enc_in, d_enc_out, nullptr, nullptr, nlines, enc_payload_bytes, nullptr, 0, nullptr,
                      nullptr, te, 1, enc_first, enc_stride, &ep);
    if (st) return st;
    const Shape sh = wave_shape(ctx, nlines / 64, kEncThreads);
    const int grid = std::min(sh.grid, enc_grid_cap(ctx));
    if (sh.threads != kDecThreads) return sequential();
    // The rest of the encrypt stream (< 1,024 payloads) first, as the strided entry point runs it.
    if (nlines < enc_npayloads) {
        st = encrypt_common(ctx, d_enc_in, d_enc_out, nullptr, nullptr, enc_npayloads - nlines, enc_payload_bytes,
                            nullptr, 0, nullptr, nullptr, s, te, 1, enc_first + nlines * enc_stride, enc_stride);
        if (st) return st;
    }
    DecPlan dp;
    st = dec_plan(ctx, d_dec_in, d_dec_out, dec_npayloads, dec_payload_bytes, nullptr, 0, nullptr, nullptr, s, td, 1,
                  dec_first, dec_stride, (int)ctx->duplex_dyn_pct, grid, &dp);
    if (st) return st;
    if (!dp.a.dyn) {  // a decrypt too short for a pool: the two launches
        CY_TRY(launch_encrypt_lines(ep.a, grid, kEncThreads, s));
        CY_TRY(launch_decrypt_flat(dp.a, dp.grid, s));
        return note_key_use(ctx, te, s);
    }
    DuplexArgs x;
    x.e = ep.a;
    x.d = dp.a;
    CY_TRY(launch_duplex_lines(x, grid, s));
    return note_key_use(ctx, te, s);
}

// Duplex of two ragged relay streams (r06): the encrypt of a stream of few,
// long payloads (0xFF00-B chunks: the quad kernel, bound by its chains'
// latency) leaves most of the chip's LDS idle.  It runs packed
// (16 waves per workgroup, on as few CUs as hold them) on `stream` while the
// decrypt runs on the context's second stream, joined back into `stream`:
// the decrypt takes the CUs the encrypt leaves.  Results as
// cyaes_gpu_encrypt_ragged(enc, key row enc_key) then
// cyaes_gpu_decrypt_ragged(dec, key row dec_key); other shapes run as those two
// calls in that order.
// The two ragged halves (validated), concurrently when the encrypt would run
// on the quad kernel, else in order on `s`.  te / td: the key tables
// (te_keys / td_keys rows) the halves' key index arrays select from (nullptr
// arrays: row 0).
static int duplex_ragged_impl(cyaes_gpu* ctx, const uint8_t* e_in, uint8_t* e_out, const uint64_t* e_off,
                              const uint32_t* e_nb, uint64_t ne, const uint32_t* e_kidx, const uint8_t* d_in,
                              uint8_t* d_out, const uint64_t* d_off, const uint32_t* d_nb, uint64_t nd,
                              const uint32_t* d_kidx, const uint32_t* te, uint32_t te_keys, const uint32_t* td,
                              uint32_t td_keys, hipStream_t s, bool dec_small = false) {
    // dec_small (the caller knows the decrypt is short beside the encrypt's
    // longest chain): side by side only when packing leaves the encrypt's
    // waves per CU as they are (few chains), since a denser encrypt runs
    // ~9 % longer.
    const uint64_t qwaves = (4 * ne + 63) / 64, cus = (uint64_t)std::max(1, ctx->num_cus);
    const uint64_t ewgs = (uint64_t)std::max(1, packed_enc_wgs(ctx, ne));
    const bool denser = (qwaves + ewgs - 1) / ewgs > (qwaves + cus - 1) / cus;
    const bool concurrent =
        ne && nd && !ctx->duplex_off && ragged_encrypt_is_quad(ctx, ne) && !(dec_small && denser);
    if (!concurrent) {
        if (ne) {
            const int st = encrypt_common(ctx, e_in, e_out, e_off, e_nb, ne, 0, e_kidx, 0, nullptr, nullptr, s, te,
                                          te_keys);
            if (st) return st;
        }
        return nd ? decrypt_ragged(ctx, d_in, d_out, d_off, d_nb, nd, d_kidx, 0, nullptr, nullptr, s, td, td_keys)
                  : CYAES_OK;
    }
    hipStream_t side;
    {
        std::lock_guard<std::mutex> lk(ctx->side_mu);
        if (!ctx->side) CY_TRY(hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
        side = ctx->side;
    }
    hipEvent_t fork = nullptr, join = nullptr;
    hipError_t e = hipEventCreateWithFlags(&fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&join, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(fork, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(side, fork, 0);  // the decrypt starts after the caller's earlier work
    int st = map_err(e);
    if (st == CYAES_OK)
        st = encrypt_common(ctx, e_in, e_out, e_off, e_nb, ne, 0, e_kidx, 0, nullptr, nullptr, s, te, te_keys, 0, 0,
                            /*pack*/ true);
    // The decrypt's workgroups (persistent) take only the CUs the encrypt's
    // leave: whichever queue the dispatcher serves first, every workgroup of
    // both launches is resident at once (a decrypt holding all CUs would
    // otherwise start the encrypt's chains only as its pool drains).
    const int dec_free = std::max(1, ctx->num_cus) - packed_enc_wgs(ctx, ne);
    const int dec_grid = std::max(ctx->dup_min_dec_wgs, dec_free / kDupUnit * kDupUnit);
    if (st == CYAES_OK)
        st = decrypt_ragged(ctx, d_in, d_out, d_off, d_nb, nd, d_kidx, 0, nullptr, nullptr, side, td, td_keys,
                            dec_grid);
    // join: the caller's stream waits for the decrypt (also on failure, for what was queued)
    if (join) {
        e = hipEventRecord(join, side);
        if (e == hipSuccess) e = hipStreamWaitEvent(s, join, 0);
        if (st == CYAES_OK) st = map_err(e);
    }
    if (fork) (void)hipEventDestroy(fork);
    if (join) (void)hipEventDestroy(join);
    return st;
}

int cyaes_gpu_duplex_ragged(cyaes_gpu* ctx, const uint8_t* d_enc_in, uint8_t* d_enc_out, const uint64_t* d_enc_offsets,
                            const uint32_t* d_enc_nbytes, uint64_t enc_npayloads, uint32_t enc_key,
                            const uint8_t* d_dec_in, uint8_t* d_dec_out, const uint64_t* d_dec_offsets,
                            const uint32_t* d_dec_nbytes, uint64_t dec_npayloads, uint32_t dec_key, void* stream) {
    if (!ctx) return CYAES_EINVAL;
    const bool has_e = enc_npayloads != 0, has_d = dec_npayloads != 0;
    if (has_e && (!d_enc_offsets || !d_enc_nbytes || !ragged_args_ok(ctx, d_enc_in, d_enc_out, nullptr, nullptr)))
        return CYAES_EINVAL;
    if (has_d && (!d_dec_offsets || !d_dec_nbytes || !ragged_args_ok(ctx, d_dec_in, d_dec_out, nullptr, nullptr)))
        return CYAES_EINVAL;
    if ((has_e && enc_key >= ctx->nkeys) || (has_d && dec_key >= ctx->nkeys)) return CYAES_ERANGE;
    if (!has_e && !has_d) return CYAES_OK;
    DeviceGuard g(ctx->device);
    return duplex_ragged_impl(ctx, d_enc_in, d_enc_out, d_enc_offsets, d_enc_nbytes, enc_npayloads, nullptr, d_dec_in,
                              d_dec_out, d_dec_offsets, d_dec_nbytes, dec_npayloads, nullptr,
                              ctx->d_keys + (uint64_t)enc_key * kSchedWords, 1,
                              ctx->d_keys + (uint64_t)dec_key * kSchedWords, 1, (hipStream_t)stream);
}

int cyaes_gpu_check(cyaes_gpu* ctx) {
    if (!ctx) return CYAES_EINVAL;
    DeviceGuard g(ctx->device);
    // Every stream this context's batches ran on (the caller's, the drop-in's,
    // the host pipe's, the batcher's): the whole device, so an asynchronous
    // fault is charged to the call that checks after it.
    CY_TRY(hipDeviceSynchronize());
    CY_TRY(hipGetLastError());
    uint32_t status = 0;
    CY_TRY(hipMemcpy(&status, ctx->d_status, 4, hipMemcpyDeviceToHost));
    if (status) {
        CY_TRY(hipMemset(ctx->d_status, 0, 4));
        return CYAES_ERANGE;
    }
    return CYAES_OK;
}

int cyaes_gpu_check_stream(cyaes_gpu* ctx, void* stream) {
    if (!ctx) return CYAES_EINVAL;
    DeviceGuard g(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    uint32_t status = 0;
    // All on `stream`: a copy on the null stream would wait for every blocking stream.
    CY_TRY(hipMemcpyAsync(&status, ctx->d_status, 4, hipMemcpyDeviceToHost, s));
    CY_TRY(hipStreamSynchronize(s));
    if (status) {
        CY_TRY(hipMemsetAsync(ctx->d_status, 0, 4, s));
        CY_TRY(hipStreamSynchronize(s));
        return CYAES_ERANGE;
    }
    return CYAES_OK;
}

int cyaes_gpu_fill_synthetic(uint8_t* d_buf, uint64_t p0, uint64_t npayloads, uint32_t payload_bytes, uint64_t seed,
                             void* stream) {
    if (!d_buf || payload_bytes % 8) return CYAES_EINVAL;
    if (npayloads == 0 || payload_bytes == 0) return CYAES_OK;
    return map_err(launch_fill_synthetic(d_buf, p0, npayloads, payload_bytes, seed, (hipStream_t)stream));
}

int cyaes_gpu_digest(const uint8_t* d_buf, uint64_t nbytes, uint64_t out[2], void* stream) {
    if (!out || nbytes % 8 || (nbytes && !d_buf)) return CYAES_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    unsigned long long* d_out = nullptr;
    CY_TRY(hipMalloc(reinterpret_cast<void**>(&d_out), 16));
    hipError_t e = hipMemsetAsync(d_out, 0, 16, s);
    if (e == hipSuccess && nbytes) e = launch_digest(d_buf, nbytes / 8, d_out, s);
    unsigned long long h[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpyAsync(h, d_out, 16, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(d_out);
    if (e != hipSuccess) return map_err(e);
    out[0] = h[0];
    out[1] = h[1];
    return CYAES_OK;
}

}  // extern "C"

// The batcher's two directions of one batch (cyaes_batcher.cpp launch): the
// SEAL / ENCRYPT list and the OPEN / DECRYPT list over one stage, disjoint
// payloads, per-request key rows of one table.
int cyaes::ragged_duplex_batch(cyaes_gpu* ctx, const uint32_t* d_table, uint32_t table_keys, uint8_t* data,
                               const uint64_t* e_off, const uint32_t* e_nb, uint64_t ne, const uint32_t* e_kidx,
                               const uint64_t* d_off, const uint32_t* d_nb, uint64_t nd, const uint32_t* d_kidx,
                               hipStream_t stream, bool dec_small) {
    if (!ctx || !d_table || (ne && (!e_off || !e_nb)) || (nd && (!d_off || !d_nb)) ||
        !ragged_args_ok(ctx, data, data, nullptr, nullptr))
        return CYAES_EINVAL;
    if (!ne && !nd) return CYAES_OK;
    DeviceGuard g(ctx->device);
    return duplex_ragged_impl(ctx, data, data, e_off, e_nb, ne, e_kidx, data, data, d_off, d_nb, nd, d_kidx, d_table,
                              table_keys, d_table, table_keys, stream, dec_small);
}

// ---- host-memory drop-in (Rijndael::encrypt / decrypt) --------------------
// Every call is one CBC chain (cyr_rijndael.cpp:588-635), synchronous, and a
// lone chain on a GPU is pure latency (~50 us for 1,472 B).  The relay calls
// Rijndael from one looper thread per core (relay_local.cpp:475), so calls
// overlap: they are combined.  A call queues itself; if no batch is running
// it becomes the leader, takes every queued call (its own included) and runs
// them as one ragged batch -- one H2D of [schedules | IVs | lists | data],
// one ragged encrypt and one ragged decrypt with per-call keys and IVs, one
// D2H -- then wakes the others.  Calls that arrive meanwhile wait and go in
// the next batch.  A single thread pays no delay: its call leads at once.
namespace {

struct DropInCall {
    bool decrypt;
    const cyaes_key* key;
    const uint8_t* in;
    uint8_t* out;
    uint32_t size;
    uint8_t* iv;  // nullable, in/out
    int status = CYAES_OK;
    bool done = false;
};

// Staging of one batch in flight.  Two slots: while one batch runs on the
// GPU the next leader gathers and launches the calls queued meanwhile, so
// latency-bound batches (a few chains each) overlap on the device.
struct DropInSlot {
    bool busy = false;
    hipStream_t stream = nullptr;
    uint8_t* pinned = nullptr;
    uint64_t pinned_cap = 0;
    uint8_t* d_buf = nullptr;
    uint64_t d_cap = 0;
};
constexpr int kDropInSlots = 2;

struct DropIn {
    std::mutex mu;  // guards pending, slot ownership and init; a leader works on its slot without it
    std::condition_variable cv;
    std::vector<DropInCall*> pending;
    cyaes_gpu* ctx = nullptr;
    DropInSlot slots[kDropInSlots];
    uint64_t batches = 0, calls = 0;  // combined batches and the calls they carried (debugging)
};

DropIn& dropin() {
    static DropIn d;
    return d;
}

int dropin_init(DropIn& d) {  // under d.mu
    if (d.ctx) return CYAES_OK;
    const char* env = getenv("CYAES_DEVICE");
    cyaes_gpu* ctx = nullptr;
    int st = cyaes_gpu_create(env ? atoi(env) : 0, &ctx);
    if (st) return st;
    DeviceGuard g(ctx->device);
    for (DropInSlot& sl : d.slots) {
        const hipError_t e = hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            for (DropInSlot& s2 : d.slots)
                if (s2.stream) (void)hipStreamDestroy(s2.stream), s2.stream = nullptr;
            cyaes_gpu_destroy(ctx);
            return map_err(e);
        }
    }
    d.ctx = ctx;
    return CYAES_OK;
}

// Grows geometrically: hipHostFree / hipFree synchronise, so a run of
// slightly growing calls must not reallocate every time.
int dropin_reserve(DropInSlot& d, uint64_t host_bytes, uint64_t dev_bytes) {
    if (d.pinned_cap < host_bytes) {
        const uint64_t cap = std::max<uint64_t>(host_bytes, 2 * d.pinned_cap);
        if (d.pinned) CY_TRY(hipHostFree(d.pinned));
        d.pinned = nullptr;
        d.pinned_cap = 0;
        CY_TRY(hipHostMalloc(reinterpret_cast<void**>(&d.pinned), cap, hipHostMallocDefault));
        d.pinned_cap = cap;
    }
    if (d.d_cap < dev_bytes) {
        const uint64_t cap = std::max<uint64_t>(dev_bytes, 2 * d.d_cap);
        if (d.d_buf) CY_TRY(hipFree(d.d_buf));
        d.d_buf = nullptr;
        d.d_cap = 0;
        CY_TRY(hipMalloc(reinterpret_cast<void**>(&d.d_buf), cap));
        d.d_cap = cap;
    }
    return CYAES_OK;
}

// Runs a batch of calls (leader, without the lock).  Image, host and device:
//   [schedules n x 352][IV in n x 16][offsets n x 8][nbytes n x 4][key index n x 4] | [data in]
// encrypt calls first, then decrypt calls; device adds [data out] and [IV out n x 16].
int dropin_batch(cyaes_gpu* ctx, DropInSlot& d, const std::vector<DropInCall*>& calls) {
    int st = CYAES_OK;
    DeviceGuard g(ctx->device);
    std::vector<DropInCall*> order;  // encrypt calls, then decrypt calls
    order.reserve(calls.size());
    for (DropInCall* c : calls)
        if (!c->decrypt) order.push_back(c);
    const size_t nenc = order.size();
    for (DropInCall* c : calls)
        if (c->decrypt) order.push_back(c);
    const uint64_t n = order.size();
    const uint64_t o_sched = 0, o_iv = n * 352, o_off = o_iv + n * 16, o_nb = o_off + n * 8, o_kid = o_nb + n * 4;
    const uint64_t o_data = (o_kid + n * 4 + 255) & ~uint64_t(255);
    uint64_t data = 0;
    for (DropInCall* c : order) data += c->size;
    const uint64_t o_out = (o_data + data + 255) & ~uint64_t(255);
    const uint64_t o_ivout = o_out + data;  // right after the results: one D2H brings both back
    st = dropin_reserve(d, o_data + data + n * 16, o_ivout + n * 16);
    if (st) return st;
    uint8_t* h = d.pinned;
    uint64_t* offs = reinterpret_cast<uint64_t*>(h + o_off);
    uint32_t* nbs = reinterpret_cast<uint32_t*>(h + o_nb);
    uint32_t* kid = reinterpret_cast<uint32_t*>(h + o_kid);
    uint64_t pos = 0;
    for (uint64_t i = 0; i < n; i++) {
        const DropInCall* c = order[i];
        to_device_schedule(*c->key, reinterpret_cast<uint32_t*>(h + o_sched + 352 * i));
        memcpy(h + o_iv + 16 * i, c->iv ? c->iv : cyaes_default_iv(), 16);
        offs[i] = pos;
        nbs[i] = c->size;
        kid[i] = (uint32_t)i;
        memcpy(h + o_data + pos, c->in, c->size);
        pos += c->size;
    }
    CY_TRY(hipMemcpyAsync(d.d_buf, h, o_data + data, hipMemcpyHostToDevice, d.stream));
    const uint32_t* table = reinterpret_cast<const uint32_t*>(d.d_buf + o_sched);
    auto dptr = [&](uint64_t o) { return d.d_buf + o; };
    // Each direction: calls of one size (the usual relay case, and any single
    // call) run as a uniform batch -- the flat decrypt spreads even one
    // payload over the whole GPU -- mixed sizes as a ragged one.
    for (int dir = 0; dir < 2; dir++) {
        const uint64_t b0 = dir ? nenc : 0, b1 = dir ? n : nenc;
        if (b1 == b0) continue;
        bool same = true;
        for (uint64_t i = b0 + 1; i < b1; i++) same = same && order[i]->size == order[b0]->size;
        const uint8_t* in = dptr(o_data) + offs[b0];
        uint8_t* out = dptr(o_out) + offs[b0];
        const uint32_t* kidx = reinterpret_cast<const uint32_t*>(dptr(o_kid)) + b0;
        const uint8_t* ivi = dptr(o_iv) + 16 * b0;
        uint8_t* ivo = dptr(o_ivout) + 16 * b0;
        if (same && dir)
            st = decrypt_uniform(ctx, in, out, b1 - b0, order[b0]->size, kidx, 0, ivi, ivo, d.stream, table,
                                 (uint32_t)n);
        else if (same)
            st = encrypt_common(ctx, in, out, nullptr, nullptr, b1 - b0, order[b0]->size, kidx, 0, ivi, ivo,
                                d.stream, table, (uint32_t)n);
        else if (dir)
            st = decrypt_ragged(ctx, dptr(o_data), dptr(o_out), reinterpret_cast<const uint64_t*>(dptr(o_off)) + b0,
                                reinterpret_cast<const uint32_t*>(dptr(o_nb)) + b0, b1 - b0, kidx, 0, ivi, ivo,
                                d.stream, table, (uint32_t)n);
        else
            st = encrypt_common(ctx, dptr(o_data), dptr(o_out), reinterpret_cast<const uint64_t*>(dptr(o_off)) + b0,
                                reinterpret_cast<const uint32_t*>(dptr(o_nb)) + b0, b1 - b0, 0, kidx, 0, ivi, ivo,
                                d.stream, table, (uint32_t)n);
        if (st) return st;
    }
    // results and final chains come back over the input image (no longer needed)
    CY_TRY(hipMemcpyAsync(h + o_data, dptr(o_out), data + n * 16, hipMemcpyDeviceToHost, d.stream));
    CY_TRY(hipStreamSynchronize(d.stream));
    const uint8_t* ivs = h + o_data + data;
    for (uint64_t i = 0; i < n; i++) {
        DropInCall* c = order[i];
        memcpy(c->out, h + o_data + offs[i], c->size);
        if (c->iv) memcpy(c->iv, ivs + 16 * i, 16);  // cyr_rijndael.cpp:607-608,633-634
    }
    return CYAES_OK;
}

// One combined call of at most dropin_piece() bytes.
int dropin_one(bool decrypt, const cyaes_key* key, const uint8_t* in, uint8_t* out, size_t size, uint8_t* iv) {
    DropIn& d = dropin();
    DropInCall me{decrypt, key, in, out, (uint32_t)size, iv};
    std::unique_lock<std::mutex> lk(d.mu);
    const int ist = dropin_init(d);
    if (ist) return ist;
    d.pending.push_back(&me);
    while (!me.done) {
        DropInSlot* slot = nullptr;
        for (DropInSlot& sl : d.slots)
            if (!sl.busy) {
                slot = &sl;
                break;
            }
        if (!slot || d.pending.empty()) {  // both slots in flight, or this call already taken by a leader
            d.cv.wait(lk);
            continue;
        }
        slot->busy = true;  // lead: take every queued call (this one, if still queued, included)
        std::vector<DropInCall*> batch;
        batch.swap(d.pending);
        lk.unlock();
        int st;
        try {
            st = dropin_batch(d.ctx, *slot, batch);
        } catch (const std::bad_alloc&) {  // the slot and the waiters must still be released
            st = CYAES_ENOMEM;
        }
        // A batch that failed part-way may still have copies in flight from the
        // slot's pinned image: drain them before another leader refills it.
        if (st && slot->stream) (void)hipStreamSynchronize(slot->stream);
        lk.lock();
        for (DropInCall* c : batch) {
            c->status = st;
            c->done = true;
        }
        d.batches++;
        d.calls += batch.size();
        slot->busy = false;
        d.cv.notify_all();
    }
    return me.status;
}

// Bytes per combined call (a batch's sizes are 32-bit); env CYAES_DROPIN_PIECE
// (a multiple of 16) lowers it so tests can reach the piece path cheaply.
uint64_t dropin_piece() {
    static const uint64_t piece = [] {
        const char* e = getenv("CYAES_DROPIN_PIECE");
        const uint64_t v = e ? strtoull(e, nullptr, 10) : 0;
        return (v >= 16 && v % 16 == 0 && v <= (1ull << 31)) ? v : (1ull << 31);
    }();
    return piece;
}

// Rijndael::encrypt / decrypt (cyr_rijndael.cpp:588-635).  The reference
// asserts size % 16 == 0 and input != NULL (its typo `input && input`,
// :590-591); size == 0 never enters its loop, whatever the pointers.  Calls
// above dropin_piece() run as consecutive pieces of one CBC chain: the final
// chain of a piece (for decrypt its last ciphertext block, read before an
// in-place piece overwrites it) is the IV of the next.
int dropin_run(bool decrypt, const cyaes_key* key, const uint8_t* in, uint8_t* out, size_t size, uint8_t* iv) {
    if (size % 16) return CYAES_EINVAL;
    if (size == 0) return CYAES_OK;  // no-op, IV unchanged (cyr_rijndael.cpp:600 loop never runs)
    if (!key || !in || !out) return CYAES_EINVAL;
    const uint64_t piece = dropin_piece();
    if (size <= piece) return dropin_one(decrypt, key, in, out, size, iv);
    uint8_t chain[16];
    memcpy(chain, iv ? iv : cyaes_default_iv(), 16);
    for (uint64_t off = 0; off < size; off += piece) {
        const int st = dropin_one(decrypt, key, in + off, out + off, std::min<uint64_t>(piece, size - off), chain);
        if (st) return st;
    }
    if (iv) memcpy(iv, chain, 16);  // cyr_rijndael.cpp:607-608, 633-634
    return CYAES_OK;
}

}  // namespace

extern "C" {

int cyaes_cbc_encrypt(const cyaes_key* key, const uint8_t* in, uint8_t* out, size_t size, uint8_t* iv) {
    return dropin_run(false, key, in, out, size, iv);
}

int cyaes_cbc_decrypt(const cyaes_key* key, const uint8_t* in, uint8_t* out, size_t size, uint8_t* iv) {
    return dropin_run(true, key, in, out, size, iv);
}

}  // extern "C"

// ---- host-resident batches streamed through the device --------------------
// The relay path starts and ends in host memory.  Three
// streams -- upload, compute, download -- and a ring of kSlots device slot
// pairs: chunk i uses slot i % kSlots; its upload waits for the kernel of
// chunk i - kSlots (slot input free), its kernel for its upload and for the
// download of chunk i - kSlots (slot output free).  Both copy directions then
// run back to back and overlap each other and the kernels.
struct HostPipe {
    static constexpr int kSlots = 3;
    int device = 0;
    hipStream_t up = nullptr, comp = nullptr, down = nullptr;
    hipEvent_t ev_up[kSlots] = {}, ev_comp[kSlots] = {}, ev_down[kSlots] = {};
    uint8_t* d_in[kSlots] = {};
    uint8_t* d_out[kSlots] = {};
    uint64_t cap = 0;
    // Pinned staging for caller ranges that are bounced instead of registered
    // (HostPin): created on first use, kBounceChunk bytes per slot.
    uint8_t* h_stage[kSlots] = {};
    uint64_t stage_cap = 0;
};
constexpr uint64_t kBounceChunk = 32ull << 20;

static void destroy_pipe(HostPipe* p) {
    if (!p) return;
    for (int i = 0; i < HostPipe::kSlots; i++) {
        (void)hipFree(p->d_in[i]);
        (void)hipFree(p->d_out[i]);
        if (p->ev_up[i]) (void)hipEventDestroy(p->ev_up[i]);
        if (p->ev_comp[i]) (void)hipEventDestroy(p->ev_comp[i]);
        if (p->ev_down[i]) (void)hipEventDestroy(p->ev_down[i]);
    }
    for (int i = 0; i < HostPipe::kSlots; i++)
        if (p->h_stage[i]) (void)hipHostFree(p->h_stage[i]);
    for (hipStream_t s : {p->up, p->comp, p->down})
        if (s) (void)hipStreamDestroy(s);
    delete p;
}

namespace {

int pipe_ready(cyaes_gpu* ctx, uint64_t slot_bytes) {
    if (!ctx->pipe) {
        HostPipe* p = new HostPipe();
        p->device = ctx->device;
        ctx->pipe = p;
        for (hipStream_t* s : {&p->up, &p->comp, &p->down}) CY_TRY(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
        for (int i = 0; i < HostPipe::kSlots; i++) {
            CY_TRY(hipEventCreateWithFlags(&p->ev_up[i], hipEventDisableTiming));
            CY_TRY(hipEventCreateWithFlags(&p->ev_comp[i], hipEventDisableTiming));
            CY_TRY(hipEventCreateWithFlags(&p->ev_down[i], hipEventDisableTiming));
        }
    }
    HostPipe* p = ctx->pipe;
    if (p->cap < slot_bytes) {
        for (hipStream_t s : {p->up, p->comp, p->down}) CY_TRY(hipStreamSynchronize(s));  // the slots' only users
        for (int i = 0; i < HostPipe::kSlots; i++) {
            (void)hipFree(p->d_in[i]);
            (void)hipFree(p->d_out[i]);
            p->d_in[i] = p->d_out[i] = nullptr;
        }
        p->cap = 0;
        for (int i = 0; i < HostPipe::kSlots; i++) {
            CY_TRY(hipMalloc(reinterpret_cast<void**>(&p->d_in[i]), slot_bytes));
            CY_TRY(hipMalloc(reinterpret_cast<void**>(&p->d_out[i]), slot_bytes));
        }
        p->cap = slot_bytes;
    }
    return CYAES_OK;
}

int stage_ready(HostPipe* p, uint64_t bytes) {
    if (p->stage_cap >= bytes) return CYAES_OK;
    for (int i = 0; i < HostPipe::kSlots; i++) {
        if (p->h_stage[i]) CY_TRY(hipHostFree(p->h_stage[i]));  // (the pipe's streams are idle between calls)
        p->h_stage[i] = nullptr;
    }
    p->stage_cap = 0;
    for (int i = 0; i < HostPipe::kSlots; i++)
        CY_TRY(hipHostMalloc(reinterpret_cast<void**>(&p->h_stage[i]), bytes, hipHostMallocDefault));
    p->stage_cap = bytes;
    return CYAES_OK;
}

// A caller's host range for the duration of one host batch (cyaes_pins.cpp).
// Registered as its exact bytes when no page of it is registered by anyone;
// used as it is when it lies inside one registration of another owner
// (hipHostMalloc, the caller's own hipHostRegister); otherwise -- pages shared
// with another registration, such as the other buffer of this call on a
// shared heap page -- it is not registered at all and its chunks are bounced
// through the pipe's pinned staging slots (direct == false).  r04's two
// illegal-address faults are the reason nothing is registered over anyone's
// pages any more.
struct HostPin {
    PinHold h;
    bool direct = false;  // DMA straight from / to the caller's memory
    void acquire(const void* p, uint64_t bytes) {
        // Any failure to register (a conflict, a pinning limit) bounces.
        direct = pin_acquire((uintptr_t)p, (uintptr_t)p + bytes, PinMode::kExclusive, &h) == CYAES_OK;
    }
    int release() {
        direct = false;
        return pin_release(&h);
    }
    ~HostPin() { (void)pin_release(&h); }  // (early returns; the explicit release reports the status)
};

struct PipeDrain {
    HostPipe* p;
    ~PipeDrain() {
        for (hipStream_t s : {p->up, p->comp, p->down}) (void)hipStreamSynchronize(s);
    }
};

int host_batch(cyaes_gpu* ctx, bool decrypt, const uint8_t* h_in, uint8_t* h_out, uint64_t npayloads,
               uint32_t payload_bytes, uint32_t ppk, uint64_t chunk_bytes) {
    if (!ctx || !h_in || !h_out || payload_bytes % 16) return CYAES_EINVAL;
    if (npayloads == 0 || payload_bytes == 0) return CYAES_OK;
    if (ctx->nkeys == 0) return CYAES_ERANGE;
    if (ppk && (npayloads - 1) / ppk >= ctx->nkeys) return CYAES_ERANGE;
    if (npayloads > UINT64_MAX / payload_bytes) return CYAES_EINVAL;
    DeviceGuard g(ctx->device);
    if (!g.ok) return CYAES_EDEVICE;
    if (chunk_bytes == 0) chunk_bytes = 256ull << 20;
    const uint64_t total = npayloads * payload_bytes;
    const bool inplace = h_out == h_in;
    HostPin pin_in, pin_out;
    pin_in.acquire(h_in, total);
    if (!inplace) pin_out.acquire(h_out, total);
    const bool bounce_in = !pin_in.direct, bounce_out = inplace ? bounce_in : !pin_out.direct;
    if (bounce_in || bounce_out) chunk_bytes = std::min(chunk_bytes, kBounceChunk);
    // Chunks hold whole payloads, and whole sessions when keys are per session,
    // so chunk c starts at session c0 / ppk and runs under that table slice.
    uint64_t cp = std::max<uint64_t>(1, chunk_bytes / payload_bytes);
    if (ppk) cp = std::max<uint64_t>(ppk, cp / ppk * ppk);
    cp = std::min(cp, npayloads);
    int st = pipe_ready(ctx, cp * payload_bytes);
    if (st) return st;
    HostPipe* p = ctx->pipe;
    if (bounce_in || bounce_out) {
        st = stage_ready(p, cp * payload_bytes);
        if (st) return st;
    }
    // Declared after the pins, so destroyed before them: on every return,
    // early ones included, the copies queued from and to the caller's pages
    // (and the staging slots) have finished before the pins are released.
    PipeDrain drain{p};
    // Chunk i's output, bounced: copied out of its staging slot once its download is done.
    auto bounce_out_chunk = [&](uint64_t i) -> int {
        const int s = (int)(i % HostPipe::kSlots);
        const uint64_t c0 = i * cp, n = std::min(cp, npayloads - c0);
        CY_TRY(hipEventSynchronize(p->ev_down[s]));
        memcpy(h_out + c0 * payload_bytes, p->h_stage[s], n * payload_bytes);
        return CYAES_OK;
    };
    const uint64_t nchunks = (npayloads + cp - 1) / cp;
    for (uint64_t i = 0; i < nchunks; i++) {
        const int s = (int)(i % HostPipe::kSlots);
        const uint64_t c0 = i * cp, n = std::min(cp, npayloads - c0);
        const uint64_t off = c0 * payload_bytes, bytes = n * payload_bytes;
        if (i >= (uint64_t)HostPipe::kSlots && bounce_out) {
            st = bounce_out_chunk(i - HostPipe::kSlots);  // frees the staging slot, too
            if (st) return st;
        } else if (i >= (uint64_t)HostPipe::kSlots && bounce_in) {
            CY_TRY(hipEventSynchronize(p->ev_up[s]));  // the slot's previous upload has read it
        }
        if (i >= (uint64_t)HostPipe::kSlots) CY_TRY(hipStreamWaitEvent(p->up, p->ev_comp[s], 0));
        const uint8_t* src = h_in + off;
        if (bounce_in) {
            memcpy(p->h_stage[s], src, bytes);
            src = p->h_stage[s];
        }
        CY_TRY(hipMemcpyAsync(p->d_in[s], src, bytes, hipMemcpyHostToDevice, p->up));
        CY_TRY(hipEventRecord(p->ev_up[s], p->up));
        CY_TRY(hipStreamWaitEvent(p->comp, p->ev_up[s], 0));
        if (i >= (uint64_t)HostPipe::kSlots) CY_TRY(hipStreamWaitEvent(p->comp, p->ev_down[s], 0));
        const uint64_t k0 = ppk ? c0 / ppk : 0;
        const uint32_t* table = ctx->d_keys + k0 * kSchedWords;
        const uint32_t tkeys = ctx->nkeys - (uint32_t)k0;
        st = decrypt ? decrypt_uniform(ctx, p->d_in[s], p->d_out[s], n, payload_bytes, nullptr, ppk, nullptr, nullptr,
                                       p->comp, table, tkeys)
                     : encrypt_common(ctx, p->d_in[s], p->d_out[s], nullptr, nullptr, n, payload_bytes, nullptr, ppk,
                                      nullptr, nullptr, p->comp, table, tkeys);
        if (st) return st;
        CY_TRY(hipEventRecord(p->ev_comp[s], p->comp));
        CY_TRY(hipStreamWaitEvent(p->down, p->ev_comp[s], 0));
        // A bounced output lands in the slot's staging buffer, which its upload
        // has already been read from (the download waits for the kernel, which
        // waited for the upload).
        CY_TRY(hipMemcpyAsync(bounce_out ? p->h_stage[s] : h_out + off, p->d_out[s], bytes, hipMemcpyDeviceToHost,
                              p->down));
        CY_TRY(hipEventRecord(p->ev_down[s], p->down));
    }
    if (bounce_out)
        for (uint64_t i = nchunks > (uint64_t)HostPipe::kSlots ? nchunks - HostPipe::kSlots : 0; i < nchunks; i++) {
            st = bounce_out_chunk(i);
            if (st) return st;
        }
    CY_TRY(hipStreamSynchronize(p->down));
    for (hipStream_t s : {p->up, p->comp}) CY_TRY(hipStreamSynchronize(s));
    // (the drain finds the streams idle)
    const int r_out = pin_out.release();
    const int r_in = pin_in.release();
    return r_in ? r_in : r_out;
}

}  // namespace

extern "C" {

int cyaes_gpu_encrypt_host(cyaes_gpu* ctx, const uint8_t* h_in, uint8_t* h_out, uint64_t npayloads,
                           uint32_t payload_bytes, uint32_t payloads_per_key, uint64_t chunk_bytes) {
    return host_batch(ctx, false, h_in, h_out, npayloads, payload_bytes, payloads_per_key, chunk_bytes);
}

int cyaes_gpu_decrypt_host(cyaes_gpu* ctx, const uint8_t* h_in, uint8_t* h_out, uint64_t npayloads,
                           uint32_t payload_bytes, uint32_t payloads_per_key, uint64_t chunk_bytes) {
    return host_batch(ctx, true, h_in, h_out, npayloads, payload_bytes, payloads_per_key, chunk_bytes);
}

}  // extern "C"
