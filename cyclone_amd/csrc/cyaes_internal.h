// cyaes_internal.h -- shared between the gfx950 kernels (cyaes_kernels.hip,
// cyaes_enc_kernels.hip, cyaes_dec_kernels.hip; device helpers in
// cyaes_device.h) and the host runtime (cyaes_runtime.cpp).  Not part of the
// public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

struct cyaes_gpu;  // include/cyaes.h

namespace cyaes {

// Device key schedule: the reference's m_Ke / m_Kd words (cyr_rijndael.h:50,52)
// byte-swapped to little-endian so a dwordx4 load of a block is directly the
// cipher state.  88 words = 352 B per key, ek at [0,44), dk at [44,88).
constexpr int kSchedWords = 88;

// LDS images.  A row is 256 B: word A[x] in slots 0..31 and
// word B[x] in slots 32..63, one copy per bank, so lane l always reads bank
// l%32 and every T-table gather is conflict-free.  The address of (x, lane)
// is one v_perm_b32: x << 8 | (lane & 31) << 2.
//   encrypt: region 0 A = TL1, B = TL2; region 1 (+64 KiB) A = TL3, B = TL4.
//   decrypt: region 0 A = TL5, B = TL6; region 1 A = TL7, B = TL8; then, at
//            128 KiB, Si x 0x01010101 in 128-B rows (32 slots), 32 KiB.
// Region 1 is addressed through byte 2 of the lane offset register (= 1).
constexpr int kEncLdsWords = 32768;  // 128 KiB
constexpr int kDecLdsWords = 40960;  // 160 KiB: the whole LDS of a CU
constexpr int kEncTableWords = 1024; // TL1, TL2, TL3, TL4
constexpr int kDecTableWords = 768;  // TL5[256], TL7[256], SiW[256]
// Byte offsets inside the device table buffer.
constexpr int kEncTableOff = 0;
constexpr int kDecTableOff = kEncTableWords * 4;
constexpr int kSboxOff = kDecTableOff + kDecTableWords * 4;
constexpr int kSiOff = kSboxOff + 256;  // inverse S-box bytes (global-memory Si lookups, CYAES_DEC_SI_VMEM)
constexpr int kTablesBytes = kSiOff + 256;

// Workgroup shapes: 16 waves x 1 WG/CU (128 / 160 KiB LDS) for both directions.
constexpr int kEncThreads = 1024;
constexpr int kEncWgPerCu = 1;
constexpr int kDecThreads = 1024;
constexpr int kDecWgPerCu = 1;
// Uniform encrypt batches with fewer chains than this run four lanes per
// chain (k_encrypt_quad), larger ones one lane per chain (k_encrypt).  Ragged
// batches switch at kQuadRaggedFactor times the count.  It was 16 while the
// lane kernel waited for each chunk's stores before its next loads (relay
// packets, payload at packet offset 12, then took 1.80 ms per 1 M in place
// against the quad kernel's 1.50); with one prefetch path it no longer does,
// and on relay streams the lane kernel wins from 131,072 packets up (0.206 vs
// 0.223 ms; 1 M: 1.30 vs 1.51 ms) and loses below (65,536: 0.149 vs 0.114)
// (scripts/ab_ragged_switch.sh, profiles/r02/ab_ragged_switch.txt).
#ifndef CYAES_QUAD_MAX_CHAINS
#define CYAES_QUAD_MAX_CHAINS 131072
#endif
constexpr uint64_t kQuadRaggedFactor = 1;
// Decrypt: blocks per lane per step (a wave step covers 64*kDecRows blocks).
#ifndef CYAES_DEC_ROWS
#define CYAES_DEC_ROWS 4
#endif
constexpr int kDecRows = CYAES_DEC_ROWS;
// Dynamic decrypt work (DecArgs.dyn): the share of a launch's work in the
// dynamic pool (%), steps per dynamic flat-decrypt range, and the ragged
// decrypt's payload groups per wave of a full grid.
constexpr uint32_t kDecDynPct = 25;
constexpr uint64_t kDecShortSteps = 256;  // steps per wave at most for the short-launch progress divisor
constexpr uint32_t kDecRangeSteps = 4;
constexpr uint32_t kDecGroupsPerWave = 8;
// The duplex launch's decrypt: its workgroups arrive from their encrypt walks
// at different times (the encrypt's tail), so a share of the work is always
// in the dynamic pool.
constexpr uint32_t kDuplexDynPct = 25;

struct Fastdiv {  // Lemire: q = mulhi64(M, n) exact for all 32-bit n, d >= 2
    uint64_t M;
    uint32_t d;
};

inline Fastdiv make_fastdiv(uint32_t d) {
    Fastdiv f;
    f.d = d;
    f.M = d > 1 ? (~0ull / d + 1) : 0;  // d == 1 is special-cased by the device fastdiv
    return f;
}

struct KeySel {
    const uint32_t* table;     // nkeys * kSchedWords words (device)
    const uint32_t* key_idx;   // per payload (nullable)
    Fastdiv ppk;               // payloads per key (d == 0 => key 0)
    uint32_t nkeys;
};

struct EncArgs {
    const uint8_t* in;
    uint8_t* out;
    const uint64_t* offsets;  // ragged (nullable => uniform)
    const uint32_t* nbytes;
    uint64_t npayloads;
    uint32_t payload_bytes;
    KeySel keys;
    const uint8_t* iv_in;
    uint8_t* iv_out;
    const uint32_t* tables;  // kEncTableWords
    uint32_t* status;
    uint32_t run;            // uniform lane kernel: payloads per work item (> 1: k_encrypt RUNS; no IV arrays)
    uint32_t sess_payloads;  // uniform lane kernel: payloads_per_key when every wave lies in one session (SESS), else 0
    uint64_t off0, stride;   // ragged kernels, stride != 0: payload p at byte off0 + p * stride, payload_bytes each
                             // (cyaes_gpu_encrypt_strided; offsets / nbytes are not read)
    // Ragged batches by lines (r06): rest[0] counts the line-walk waves
    // (1,024-payload-group wave indices, rest[1..]) the line kernel handed back;
    // the ragged lane kernel, given rest, walks exactly those waves' payloads.
    uint32_t* rest;
};

// Per-launch decrypt scratch (DecArgs.work): words kWorkCtrOff + 64 * x are
// the ticket counters of the dynamic pools, one per XCD (a 256-B line each),
// and words kWorkLeadOff + workgroup, after all of them, the progress-feedback
// leader words, so no grid size can make the two overlap.  Per
// launch, so concurrent decrypts on different streams never share them
// (VERDICT r03, weak 7).
constexpr uint32_t kWorkCtrOff = 0;
constexpr uint32_t kXcds = 8;  // MI355X; on a chip with fewer, the spare pools are simply stolen from
constexpr uint32_t kWorkLeadOff = kWorkCtrOff + 64 * kXcds;
constexpr uint32_t dec_work_words(uint32_t grid) { return kWorkLeadOff + grid; }

struct DecArgs {
    const uint8_t* in;
    uint8_t* out;
    const uint64_t* offsets;  // ragged kernel only
    const uint32_t* nbytes;
    uint64_t npayloads;
    uint64_t nblocks;         // flat kernel: total blocks = npayloads * bpp
    // Work ranges (flat kernel; the ragged kernel's unit is a payload group):
    // ranges [0, nstat) are static, stat_blocks long, wave w takes range w (and
    // w + nwaves, ... when there are more); ranges [nstat, nranges) are the
    // dynamic pool (dyn), range_blocks long, handed out by per-XCD ticket
    // counters with stealing (cyaes_device.h, dyn_ticket).
    uint64_t stat_blocks;     // flat kernel: blocks per static range (a multiple of 64*kDecRows)
    uint64_t range_blocks;    // flat kernel: blocks per dynamic range (a multiple of 64*kDecRows)
    uint64_t nranges;         // flat kernel: static + dynamic ranges; ragged kernel: payload groups
    uint32_t nstat;           // static ranges / groups
    uint32_t per_xcd;         // dyn: tickets per XCD pool (ceil((nranges - nstat) / kXcds))
    uint32_t* work;           // per-launch scratch (dec_work_words, zeroed before a dyn launch): counters, progress words
    uint32_t dyn;             // 1: ranges [nstat, nranges) from the ticket pools
    uint32_t prio_short;      // flat kernel: few steps per wave, the short-launch progress divisor (kDecPrioDivShort)
    Fastdiv bpp;              // flat kernel: blocks per payload
    uint32_t step_q, step_r;  // (64*kDecRows) / bpp, % bpp
    KeySel keys;
    const uint8_t* iv_in;
    uint8_t* iv_out;
    const uint4* boundary;    // flat kernel in-place: a 32-B record per range, C[begin-1] first (nullable)
    uint32_t inplace;         // in == out: drain a step's loads before its stores
    const uint32_t* tables;   // kDecTableWords
    uint32_t* status;
    uint32_t group;           // ragged kernel: payloads per wave group (1..64)
    uint64_t sess_blocks;     // flat kernel: blocks per payloads_per_key session when a multiple of a step, else 0
    uint64_t off0, stride;    // flat kernel, stride != 0: payload p at byte off0 + p * stride (4-B aligned), else contiguous
    // Flat kernel in place, static ranges, no prepass: != 0 the launch's epoch,
    // with which the waves tag the boundary records they publish (dec_handoff,
    // cyaes_dec_body.h).
    uint64_t handoff;
    // Flat kernel, XCD-weighted static split (A/B, env CYAES_DEC_XCD_W): one
    // range per wave; the waves of workgroups b = x mod 8 take xsteps[x] steps
    // each, the slots' spans laid out in slot order.
    uint32_t xw;
    uint32_t xsteps[kXcds];
};

// The duplex launch (cyaes_duplex_kernels.hip): one grid encrypts batch e,
// then, workgroup by workgroup, decrypts batch d (unkeyed halves, no IV arrays,
// uniform contiguous batches; d.dyn on).
struct DuplexArgs {
    EncArgs e;
    DecArgs d;
};

// Launchers (cyaes_*kernels.hip).  All asynchronous on `stream`.
hipError_t launch_encrypt(const EncArgs& a, int grid, int threads, hipStream_t stream);
// Strided, unkeyed, no IV arrays, npayloads a multiple of kLinesGroup (k_encrypt_lines).
constexpr uint64_t kLinesGroup = 1024;
hipError_t launch_encrypt_lines(const EncArgs& a, int grid, int threads, hipStream_t stream);
// Ragged (lists), unkeyed, no IV arrays, npayloads a multiple of kLinesGroup,
// a.rest zeroed at [0] and room for npayloads / 64 wave indices after it.
hipError_t launch_encrypt_rag_lines(const EncArgs& a, int grid, int threads, hipStream_t stream);
// Four lanes per chain (latency-bound batches; threads a multiple of 64).
hipError_t launch_encrypt_quad(const EncArgs& a, int grid, int threads, hipStream_t stream);
hipError_t launch_decrypt_flat(const DecArgs& a, int grid, hipStream_t stream);
hipError_t launch_decrypt_ragged(const DecArgs& a, int grid, int threads, hipStream_t stream);
// The flat decrypt's per-payload-key instantiations (cyaes_ragged_kernels.hip): for launch_decrypt_flat.
void launch_decrypt_flat_keyed(const DecArgs& a, dim3 g, dim3 b, hipStream_t stream);
hipError_t launch_duplex(const DuplexArgs& x, int grid, hipStream_t stream);  // 1024-thread workgroups
// Relay streams: x.e strided, unkeyed, whole kLinesGroup groups (the lines
// walk); x.d strided (the flat kernel's STRIDED rows), dyn on.
hipError_t launch_duplex_lines(const DuplexArgs& x, int grid, hipStream_t stream);
// Before a decrypt: zeroes its work words and, for an in-place flat decrypt
// (boundary != NULL), snapshots C[begin-1] of every range that starts inside a payload.
hipError_t launch_dec_prepass(const DecArgs& a, uint32_t work_words, hipStream_t stream);
hipError_t launch_key_expand(const uint8_t* d_keys, uint32_t nkeys, const uint8_t* d_sbox,
                             uint32_t* d_sched, hipStream_t stream);
hipError_t launch_strided_lists(uint64_t* offsets, uint32_t* nbytes, uint64_t first, uint64_t stride, uint64_t n,
                                uint32_t payload_bytes, hipStream_t stream);
hipError_t launch_fill_synthetic(uint8_t* buf, uint64_t p0, uint64_t npayloads, uint32_t payload_bytes,
                                 uint64_t seed, hipStream_t stream);
hipError_t launch_digest(const uint8_t* buf, uint64_t nwords, unsigned long long* out2, hipStream_t stream);
// Variant builds: read and clear the debug records of the encrypt / decrypt
// kernel TUs (CYAES_BOUNDS_CHECK: 4 words + the per-position miss counts;
// CYAES_CLOCK_PROBE: 8 words).  cyaes_debug_bounds / _probe sum them.
int bounds_read_enc(unsigned long long* rec4, unsigned int* lines);
int bounds_read_dec(unsigned long long* rec4, unsigned int* lines);
int bounds_read_dup(unsigned long long* rec4, unsigned int* lines);
int bounds_read_rag(unsigned long long* rec4, unsigned int* lines);
int probe_read_enc(unsigned long long* out8);
int probe_read_dec(unsigned long long* out8);
int probe_read_dup(unsigned long long* out8);
int probe_read_rag(unsigned long long* out8);
int timeline_read_dup(int kind, uint4* out);
int timeline_read_enc(int kind, uint4* out);
int timeline_read_dec(int kind, uint4* out);
int timeline_read_rag(int kind, uint4* out);

// Batching adapter request descriptor (cyaes_batcher.cpp builds them in pinned
// memory, cyaes_batch_kernels.hip reads them).  src / dst are DEVICE
// addresses: a registered host packet pool (mapped) or the batcher's bounce
// buffer.  Op codes = CYAES_OP_* (cyaes_batch.h).
constexpr uint32_t kOpEncrypt = 0, kOpDecrypt = 1, kOpRelaySeal = 2, kOpRelayOpen = 3;
struct BatchDesc {
    uint64_t src;    // ENCRYPT/DECRYPT: input; SEAL: chunk; OPEN: packet
    uint64_t dst;    // ENCRYPT/DECRYPT: output; SEAL: packet out; OPEN: the packet (in place)
    uint32_t size;   // ENCRYPT/DECRYPT: bytes; SEAL: chunk bytes; OPEN: packet bytes
    uint32_t crypt;  // bytes en/decrypted (SEAL: the chunk rounded up to 16)
    uint32_t key;    // row of the batcher's device key table
    int32_t conn;    // SEAL: RelayForwardMsg::id
    uint32_t op;
    uint32_t stage;  // byte offset of the request's data in the batch's HBM stage
};
static_assert(sizeof(BatchDesc) == 40, "BatchDesc layout");
// One kernel for both PCIe directions of the batcher's pipeline: gather of
// one batch (gdesc[0, gn) into gstage, plus the ragged lists offs / nbytes /
// kidx) and scatter of the previous one (sdesc[0, sn) out of sstage).
struct BatchMove {
    const BatchDesc* gdesc;
    uint32_t gn, sn;
    uint8_t* gstage;
    uint64_t* offs;
    uint32_t* nbytes;
    uint32_t* kidx;
    const BatchDesc* sdesc;
    const uint8_t* sstage;
};
hipError_t launch_batch_move(const BatchMove& m, int max_waves, hipStream_t stream);

// Host runtime (cyaes_runtime.cpp): ragged batch under an explicit device key
// table of table_keys schedules (the batcher's per-batch session keys).
// key_idx (device, nullable => key 0) indexes that table.
// True when a ragged encrypt of n chains runs four lanes per chain
// (k_encrypt_quad: per-chain keys, no key waterfall, so no need to sort by key).
bool ragged_encrypt_is_quad(const cyaes_gpu* ctx, uint64_t n);
int ragged_batch(cyaes_gpu* ctx, bool decrypt, const uint32_t* d_table, uint32_t table_keys, const uint8_t* in,
                 uint8_t* out, const uint64_t* offsets, const uint32_t* nbytes, uint64_t npayloads,
                 const uint32_t* key_idx, hipStream_t stream);
// Both directions of a batcher batch over one stage (disjoint payloads): as
// ragged_batch(encrypt) then ragged_batch(decrypt), the two run side by side
// when the encrypt is a few long chains (cyaes_gpu_duplex_ragged's scheme).
int ragged_duplex_batch(cyaes_gpu* ctx, const uint32_t* d_table, uint32_t table_keys, uint8_t* data,
                        const uint64_t* e_off, const uint32_t* e_nb, uint64_t ne, const uint32_t* e_kidx,
                        const uint64_t* d_off, const uint32_t* d_nb, uint64_t nd, const uint32_t* d_kidx,
                        hipStream_t stream, bool dec_small);

// Host-memory registrations (cyaes_pins.cpp): every hipHostRegister the
// library makes, in one process-wide registry.
constexpr uintptr_t kPinPage = 4096;
constexpr int kPinConflict = 1;  // internal: pages another owner (or a host batch) holds
enum class PinMode {
    kShared,     // a batcher pool: its pages registered, shared with other pools' registrations by reference count
    kExclusive,  // a host batch's buffer: the exact byte range, on pages no other registration touches
};
struct PinHold {
    std::vector<uintptr_t> regs;  // registry entries holding the range, one reference each
    bool foreign = false;         // inside one registration of another owner: used as it is, nothing held
};
// CYAES_OK (held or foreign), kPinConflict, or an error; on failure nothing is held.
int pin_acquire(uintptr_t lo, uintptr_t hi, PinMode mode, PinHold* h);
// Drops the references; unregisters what no one holds any more.  Returns
// CYAES_EDEVICE if an unregister failed or left the runtime answering for the range.
int pin_release(PinHold* h);
// [lo, hi) of each registration held (the batcher's device-view checks).
void pin_bounds(const PinHold& h, std::vector<uintptr_t>* out);

}  // namespace cyaes
