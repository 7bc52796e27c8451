/*
 * cyaes_batch.h -- asynchronous batching adapter.
 *
 * The reference calls Rijndael::encrypt/decrypt synchronously, one relay
 * packet at a time, on each pipe's looper thread (relay_local.cpp:188-217,
 * 365; relay_server.cpp:329, 453-481).  A single packet is one CBC chain of
 * at most 4,080 blocks, so on a GPU it is all latency.  This adapter takes
 * those calls from any number of threads, coalesces whatever arrives within
 * a short window into one GPU batch and invokes each request's completion
 * callback -- where a relay would then post TcpConnection::send to its looper.
 *
 * Zero-copy packet pools: memory the caller registers once
 * (cyaes_batcher_register_pool) is read and written by the GPU itself over
 * PCIe: a batch's inputs are gathered from the pools into HBM by a kernel,
 * SEAL packets are built there, the ragged AES kernels run, and a kernel
 * scatters the outputs back into the pools.  The host copies no payload
 * byte; its per-request work is a 40-byte descriptor.  A request whose
 * buffers lie in registered pools takes this path automatically (pointer
 * submits) or explicitly (cyaes_batcher_submit_pooled, pool offsets).
 * Buffers outside every pool are copied through the batcher's pinned bounce
 * memory instead (same results, host copies in and out).
 *
 * Sessions (row 3): every request names a session slot.  A slot holds the
 * key of one relay pipe direction (relay_server.cpp:218-240 creates the
 * Rijndael pair after the DH handshake; :370-375 deletes it on close).
 * Its schedule is expanded once on open into a row of the batcher's device
 * key table; a closed slot's row is reused only after every request
 * submitted before the close has completed, so opening and closing sessions
 * never races in-flight batches.
 *
 * Request semantics = Rijndael::encrypt / decrypt (cyr_rijndael.cpp:588-635)
 * with iv == nullptr, as every relay call site passes: one CBC chain from
 * DefaultIV per request; size % 16 == 0; in == out allowed.
 * RELAY_SEAL / RELAY_OPEN are the relay's packet operations (cyaes_relay.h):
 *   SEAL: build the RELAY_FORWARD packet for a chunk (header, RelayForwardMsg,
 *         0xCE padding) and encrypt its payload (relay_local.cpp:189-206);
 *   OPEN: decrypt a received RELAY_FORWARD packet's payload in place
 *         (relay_server.cpp:329); the whole packet is read and written back,
 *         its 12 header bytes unchanged.
 *
 * Pipelining: `inflight` stages; while the GPU runs batch k the builder lays
 * out batch k+1 and the completion side runs k-1's callbacks.  Callbacks run
 * on the completion thread and the worker threads, one submitting thread's
 * requests in its submission order; they must not block on the batcher
 * (flush/destroy/unregister) themselves.
 */
#ifndef CYAES_BATCH_H
#define CYAES_BATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CYAES_OP_ENCRYPT 0
#define CYAES_OP_DECRYPT 1
#define CYAES_OP_RELAY_SEAL 2
#define CYAES_OP_RELAY_OPEN 3

typedef struct cyaes_batcher cyaes_batcher;

/* Completion: status is CYAES_OK or a CYAES_E* code (cyaes.h). */
typedef void (*cyaes_done_fn)(void* user, int status);

typedef struct cyaes_batcher_config {
    int device;               /* HIP device                                          */
    uint32_t max_batch_bytes; /* staging bytes per batch (0 => 32 MiB); caps a request */
    uint32_t max_delay_us;    /* longest a request waits for company (0 => 100 us)     */
    uint32_t inflight;        /* stages / batches in flight (0 => 3)                   */
    uint32_t workers;         /* completion-side threads: callbacks, bounce copies (0 => 4) */
    uint32_t max_sessions;    /* device key-table rows (0 => 65536)                    */
    uint32_t flags;           /* CYAES_BATCHER_POLL                                    */
} cyaes_batcher_config;

/* Completion queues instead of callbacks: with this flag a request submitted
 * with done == NULL completes into its submitting thread's queue, which the
 * thread drains with cyaes_batcher_poll -- the way a relay looper picks up its
 * finished packets on its own thread before TcpConnection::send
 * (relay_local.cpp:206-216), one lock per batch instead of one call per
 * packet.  (Without the flag, done == NULL means no notification.) */
#define CYAES_BATCHER_POLL 1u

int cyaes_batcher_create(const cyaes_batcher_config* cfg, cyaes_batcher** out);
/* Completes every submitted request, then frees everything. */
void cyaes_batcher_destroy(cyaes_batcher* b);

/* Session slots.  open returns the lowest free slot. close frees it; requests
 * already submitted under it still complete with the old key. */
int cyaes_batcher_session_open(cyaes_batcher* b, const uint8_t key[16], uint32_t* slot);
int cyaes_batcher_session_close(cyaes_batcher* b, uint32_t slot);

/* op ENCRYPT / DECRYPT: out[0, size) = CBC(in[0, size)) under the slot's key.
 * CYAES_EINVAL: size % 16, size > max_batch_bytes, NULL buffer, bad op;
 * CYAES_ERANGE: slot not open.  On an error return `done` is not called. */
int cyaes_batcher_submit(cyaes_batcher* b, int op, uint32_t slot, const uint8_t* in, uint8_t* out, size_t size,
                         cyaes_done_fn done, void* user);
/* RELAY_SEAL: packet_out receives cyaes_relay_packet_bytes(size) bytes,
 * size <= CYAES_RELAY_MAX_CHUNK. */
int cyaes_batcher_submit_seal(cyaes_batcher* b, uint32_t slot, int32_t conn_id, const uint8_t* payload,
                              uint32_t size, uint8_t* packet_out, cyaes_done_fn done, void* user);
/* RELAY_OPEN: packet holds one complete RELAY_FORWARD packet of packet_bytes
 * (= 4 + packet_size); its payload is decrypted in place. */
int cyaes_batcher_submit_open(cyaes_batcher* b, uint32_t slot, uint8_t* packet, uint32_t packet_bytes,
                              cyaes_done_fn done, void* user);

/* Bulk submit: one call for all the requests a relay looper collected in one
 * poll iteration (one shard lock for all of them).  Per request:
 *   ENCRYPT / DECRYPT: in, out, size as cyaes_batcher_submit;
 *   RELAY_SEAL: in = payload, size = chunk bytes, out = packet_out, conn_id;
 *   RELAY_OPEN: out (or in) = packet, size = packet bytes.
 * Invalid requests are skipped (their `done` is not called); status[i]
 * (nullable) receives each request's code; returns the first error or
 * CYAES_OK.  A thread's requests complete in its submission order. */
typedef struct cyaes_batch_req {
    int op;
    uint32_t slot;
    int32_t conn_id;
    const uint8_t* in;
    uint8_t* out;
    uint32_t size;
    cyaes_done_fn done;
    void* user;
} cyaes_batch_req;
int cyaes_batcher_submit_many(cyaes_batcher* b, const cyaes_batch_req* reqs, uint32_t n, int* status);

/* Packet pools.  register: pins the pages of [base, base + bytes) for the
 * device (hipHostRegister, mapped) and returns a pool id; pools may not
 * overlap (CYAES_EINVAL), at most 64 (CYAES_ENOMEM).  Pools may share a page
 * (two buffers of one heap): pages this batcher already pinned are shared and
 * stay pinned while any live pool uses them.  Memory pinned by someone else
 * (hipHostMalloc, the caller's hipHostRegister) is used as it is only if one
 * such registration holds the whole range, else CYAES_EINVAL; the device view
 * of the pool is checked to be contiguous.  unregister: waits until every
 * request submitted before the call has completed (their errors are kept for
 * the next cyaes_batcher_flush), then unpins the pages no other live pool
 * uses.  Requests may not use the pool concurrently with its unregister. */
int cyaes_batcher_register_pool(cyaes_batcher* b, void* base, size_t bytes, uint32_t* pool);
int cyaes_batcher_unregister_pool(cyaes_batcher* b, uint32_t pool);

/* Bulk submit by pool offsets (zero-copy).  Per request, as cyaes_batch_req
 * with in = pool base + in_off and out = pool base + out_off (OPEN: the packet
 * at in_off, decrypted in place; out_off ignored).  A request whose bytes do
 * not lie inside the pool is CYAES_EINVAL. */
typedef struct cyaes_pool_req {
    int op;
    uint32_t slot;
    int32_t conn_id;
    uint32_t pool;
    uint64_t in_off;
    uint64_t out_off;
    uint32_t size;
    cyaes_done_fn done;
    void* user;
} cyaes_pool_req;
int cyaes_batcher_submit_pooled(cyaes_batcher* b, const cyaes_pool_req* reqs, uint32_t n, int* status);

/* CYAES_BATCHER_POLL: pops up to max completions (user pointer, status) of
 * the calling thread's queue, oldest first (a thread's requests complete in
 * its submission order; threads that share a submission shard share a queue).
 * Returns the number popped; never blocks. */
uint32_t cyaes_batcher_poll(cyaes_batcher* b, void** users, int* status, uint32_t max);

/* Blocks until every request submitted before the call has completed
 * (callbacks returned).  Returns the first error status seen since the
 * previous flush, else CYAES_OK. */
int cyaes_batcher_flush(cyaes_batcher* b);

/* out[0..5] = requests completed, batches, payload bytes, largest batch
 * (requests), requests completed with an error, requests pending. */
int cyaes_batcher_stats(cyaes_batcher* b, uint64_t out[6]);

#ifdef __cplusplus
}
#endif

#endif /* CYAES_BATCH_H */
