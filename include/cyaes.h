/*
 * cyaes.h -- C-ABI of the MI355X-native cyCrypt AES-128-CBC path.
 *
 * Drop-in boundary for thejinchao/cyclone `cyclone::Rijndael`
 * (source/cyCrypt/crypt/cyr_rijndael.h:11-53).  The reference boundary is a
 * C++ class statically linked into libcyclone.a; this header is the flat
 * C-ABI beneath the same-shaped C++ class in <cyclone_amd/cyr_rijndael.h>.
 * Plain pointers and sizes only: no HIP or torch types.  `stream` arguments
 * are a hipStream_t passed as void* (NULL = the device's null stream).
 *
 * Semantics follow the reference exactly:
 *   - AES-128, CBC mode, no padding; size must be a multiple of 16
 *     (the reference asserts, cyr_rijndael.cpp:590-591,614-615; here
 *     CYAES_EINVAL is returned instead).  size == 0 is a no-op.
 *   - iv == NULL  => chain starts at DefaultIV (cyr_rijndael.cpp:503-504,
 *     594-598) and nothing is written back.  iv != NULL => chain starts at
 *     *iv and the final chain block (last ciphertext block) is written back
 *     (cyr_rijndael.cpp:607-608, 633-634), for encrypt and decrypt alike.
 *   - in == out (in place) is allowed (cyr_rijndael.cpp:626-629).
 * Every batch entry point treats each payload as an independent CBC chain,
 * as the relay sample does (relay_local.cpp:206,365; relay_server.cpp:329,472).
 */
#ifndef CYAES_H
#define CYAES_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CYAES_BLOCK_SIZE 16 /* Rijndael::BLOCK_SIZE, cyr_rijndael.h:14 */
#define CYAES_ROUNDS 10     /* cyr_rijndael.h:48 */

/* Status codes (the reference has none: it asserts). */
#define CYAES_OK 0
#define CYAES_EINVAL (-1)  /* NULL pointer, size % 16 != 0, bad argument   */
#define CYAES_EDEVICE (-2) /* HIP runtime / launch failure                  */
#define CYAES_ENOMEM (-3)  /* device or pinned allocation failed            */
#define CYAES_ERANGE (-4)  /* key index >= number of keys set               */
#define CYAES_ENODEV (-5)  /* no usable gfx950 device                       */

/* Expanded key: same words and layout as the reference object state
 * Rijndael::m_Ke / m_Kd (cyr_rijndael.h:48-52; big-endian packed words,
 * Kd = equivalent inverse cipher schedule). sizeof == 352. */
typedef struct cyaes_key {
    uint32_t ke[CYAES_ROUNDS + 1][4];
    uint32_t kd[CYAES_ROUNDS + 1][4];
} cyaes_key;

/* Rijndael::DefaultIV, cyr_rijndael.cpp:503-504 (bytes 00 01 .. 0f). */
const uint8_t* cyaes_default_iv(void);
const char* cyaes_strerror(int status);
const char* cyaes_version(void);

/* Rijndael::Rijndael(const BLOCK key), cyr_rijndael.cpp:507-572.
 * Host-side key schedule (setup, not the hot path). */
int cyaes_key_expand(const uint8_t key[16], cyaes_key* out);

/* ---- Host-memory drop-in (GPU-executed) -------------------------------
 * Rijndael::encrypt / Rijndael::decrypt (cyr_rijndael.cpp:588-609, 612-635)
 * on host buffers.  The call stages through pinned memory, runs the gfx950
 * kernel on the process default device (env CYAES_DEVICE, default 0) and
 * returns when the output is in host memory.  Thread-safe (calls serialise
 * on the process context).  One call = one CBC chain, so encrypt is
 * latency-bound on any device; batch through the device API for throughput. */
int cyaes_cbc_encrypt(const cyaes_key* key, const uint8_t* in, uint8_t* out, size_t size, uint8_t* iv);
int cyaes_cbc_decrypt(const cyaes_key* key, const uint8_t* in, uint8_t* out, size_t size, uint8_t* iv);

/* ---- Device context ----------------------------------------------------- */
typedef struct cyaes_gpu cyaes_gpu;

int cyaes_gpu_create(int device, cyaes_gpu** out);
/* Synchronises the device, frees the context and returns the synchronisation's
 * status: CYAES_EDEVICE if an asynchronous fault is pending (from this
 * context's work or any other on the device), else CYAES_OK.  The context is
 * freed either way. */
int cyaes_gpu_destroy(cyaes_gpu* ctx);
int cyaes_gpu_device(const cyaes_gpu* ctx);
/* Number of compute units, and workgroups the batch kernels launch per CU. */
int cyaes_gpu_num_cus(const cyaes_gpu* ctx);

/* Session-key table.  set_keys expands nkeys raw 16-byte keys on the host
 * and uploads the schedules; set_keys_device expands raw keys already in
 * device memory (e.g. just received by an RCCL broadcast) on the device.
 * Both replace the whole table.  Synchronous w.r.t. later batch calls on
 * `stream` (set_keys is fully synchronous). */
int cyaes_gpu_set_keys(cyaes_gpu* ctx, const uint8_t* keys, uint32_t nkeys);
int cyaes_gpu_set_keys_device(cyaes_gpu* ctx, const uint8_t* d_keys, uint32_t nkeys, void* stream);
/* Replaces (or appends) schedules [first, first + n) from n raw keys, growing
 * the table if needed; rows outside the range are kept.  first <= nkeys.
 * Per-session key plumbing: a relay session opens (relay_server.cpp:218-240,
 * a new Rijndael pair per DH handshake) or its slot is reused after a close
 * (relay_server.cpp:370-375).  Synchronous, like set_keys. */
int cyaes_gpu_update_keys(cyaes_gpu* ctx, uint32_t first, const uint8_t* keys, uint32_t n);
uint32_t cyaes_gpu_nkeys(const cyaes_gpu* ctx);
/* Copies schedule `index` back in reference layout (m_Ke/m_Kd). Synchronous. */
int cyaes_gpu_get_key(cyaes_gpu* ctx, uint32_t index, cyaes_key* out);

/* ---- Device batches (device pointers; asynchronous on `stream`) ---------
 * Key of payload p:  d_key_idx ? d_key_idx[p]
 *                  : payloads_per_key ? p / payloads_per_key : 0.
 * Chain input of payload p:  d_iv_in ? d_iv_in + 16*p : DefaultIV.
 * If d_iv_out != NULL the final chain block of payload p is written to
 * d_iv_out + 16*p (d_iv_out may equal d_iv_in).
 * d_in == d_out (in place) is allowed; partial overlap is undefined.
 * A d_key_idx entry >= nkeys is clamped and reported by cyaes_gpu_check.
 *
 * Uniform layout: payload p occupies bytes [p*payload_bytes, (p+1)*payload_bytes).
 * Ragged layout:  payload p occupies [d_offsets[p], d_offsets[p] + d_nbytes[p]);
 *                 sizes must be multiples of 16, offsets (and d_in/d_out)
 *                 multiples of 4, so a relay packet's payload at packet
 *                 offset 12 can be processed where it lies. */
int cyaes_gpu_encrypt_uniform(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, uint64_t npayloads,
                              uint32_t payload_bytes, const uint32_t* d_key_idx, uint32_t payloads_per_key,
                              const uint8_t* d_iv_in, uint8_t* d_iv_out, void* stream);
int cyaes_gpu_decrypt_uniform(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, uint64_t npayloads,
                              uint32_t payload_bytes, const uint32_t* d_key_idx, uint32_t payloads_per_key,
                              const uint8_t* d_iv_in, uint8_t* d_iv_out, void* stream);
int cyaes_gpu_encrypt_ragged(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, const uint64_t* d_offsets,
                             const uint32_t* d_nbytes, uint64_t npayloads, const uint32_t* d_key_idx,
                             uint32_t payloads_per_key, const uint8_t* d_iv_in, uint8_t* d_iv_out, void* stream);
int cyaes_gpu_decrypt_ragged(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, const uint64_t* d_offsets,
                             const uint32_t* d_nbytes, uint64_t npayloads, const uint32_t* d_key_idx,
                             uint32_t payloads_per_key, const uint8_t* d_iv_in, uint8_t* d_iv_out, void* stream);

/* Strided layout (a relay stream of equal packets resident in HBM):
 *                 payload p occupies [first_offset + p*stride, + payload_bytes);
 *                 first_offset, stride and d_in/d_out multiples of 4, stride >=
 *                 payload_bytes; the bytes between payloads are not touched.
 *                 The same result as a ragged batch with d_offsets[p] =
 *                 first_offset + p*stride and d_nbytes[p] = payload_bytes, without
 *                 the two lists: the relay server's received stream of MTU
 *                 packets, payload at packet offset 12, stride = packet size
 *                 (relay_server.cpp:329; cyaes_relay_stride finds it).  No IV
 *                 arrays (the relay passes iv = nullptr).  Kernel choice (results
 *                 identical): back-to-back 16-B aligned payloads run as a uniform
 *                 batch; unkeyed decrypts of >= 64-block payloads spanning < 4 GiB
 *                 run the flat decrypt's strided rows; the rest the ragged kernels. */
int cyaes_gpu_encrypt_strided(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, uint64_t first_offset,
                              uint64_t stride, uint64_t npayloads, uint32_t payload_bytes, const uint32_t* d_key_idx,
                              uint32_t payloads_per_key, void* stream);
int cyaes_gpu_decrypt_strided(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, uint64_t first_offset,
                              uint64_t stride, uint64_t npayloads, uint32_t payload_bytes, const uint32_t* d_key_idx,
                              uint32_t payloads_per_key, void* stream);

/* The batch entry points of SURVEY.md §8(b), as ragged batches with one
 * input IV per payload (d_iv: 16 B per payload, NULL => DefaultIV), key
 * d_key_idx[p] (NULL => key 0) and no IV write-back. */
int cyaes_gpu_cbc_encrypt_batch(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, const uint64_t* d_offsets,
                                const uint32_t* d_nbytes, const uint32_t* d_key_idx, const uint8_t* d_iv,
                                uint32_t npayloads, void* stream);
int cyaes_gpu_cbc_decrypt_batch(cyaes_gpu* ctx, const uint8_t* d_in, uint8_t* d_out, const uint64_t* d_offsets,
                                const uint32_t* d_nbytes, const uint32_t* d_key_idx, const uint8_t* d_iv,
                                uint32_t npayloads, void* stream);

/* ---- Duplex: one batch encrypted and another decrypted in ONE launch ------
 * The relay carries both directions of a pipe at once (relay_server.cpp:472
 * encrypts target -> tunnel while :329 decrypts tunnel -> target;
 * relay_local.cpp:206 / :365 on the client).  Same results as
 *   cyaes_gpu_encrypt_uniform(enc batch, key row enc_key)
 *   cyaes_gpu_decrypt_uniform(dec batch, key row dec_key)
 * in that order: uniform contiguous batches, one key each (a row of the key
 * table), no IV arrays (every payload a chain from DefaultIV), 16-B aligned
 * buffers, in place allowed.  One grid walks the encrypt batch and then,
 * workgroup by workgroup, the decrypt batch from a dynamic pool, so the
 * encrypt's tail (a CBC chain per lane cannot be split; the XCDs' clocks
 * differ) is filled with decrypt work instead of idling.  Halves too small to
 * fill the GPU, and batches whose bytes overlap, run as the two ordinary
 * launches.  Either half may be empty (npayloads or payload_bytes 0).
 * Errors: CYAES_EINVAL (size % 16, NULL or misaligned buffer), CYAES_ERANGE
 * (key row >= the number of keys set). */
int cyaes_gpu_duplex_uniform(cyaes_gpu* ctx, const uint8_t* d_enc_in, uint8_t* d_enc_out, uint64_t enc_npayloads,
                             uint32_t enc_payload_bytes, uint32_t enc_key, const uint8_t* d_dec_in, uint8_t* d_dec_out,
                             uint64_t dec_npayloads, uint32_t dec_payload_bytes, uint32_t dec_key, void* stream);

/* Duplex of two relay streams (strided layout, as cyaes_gpu_{en,de}crypt_strided):
 * the stream a relay end sends (encrypted, relay_local.cpp:206 /
 * relay_server.cpp:472) and the one it receives (decrypted, relay_server.cpp:329
 * / relay_local.cpp:365) in ONE launch.  Same results as
 *   cyaes_gpu_encrypt_strided(enc stream, key row enc_key)
 *   cyaes_gpu_decrypt_strided(dec stream, key row dec_key)
 * in that order (unkeyed within each half, one key row each, no IV arrays).
 * The encrypt half's whole 1,024-payload groups are read by 64-B lines, the
 * decrypt half by the flat kernel's strided rows; streams those kernels do not
 * take (short, unaligned, > 4 GiB spans, 16-B aligned back-to-back payloads)
 * and overlapping streams run as the two calls.  Errors as the strided entry
 * points; CYAES_ERANGE for a key row >= the number of keys set. */
int cyaes_gpu_duplex_strided(cyaes_gpu* ctx, const uint8_t* d_enc_in, uint8_t* d_enc_out, uint64_t enc_first_offset,
                             uint64_t enc_stride, uint64_t enc_npayloads, uint32_t enc_payload_bytes, uint32_t enc_key,
                             const uint8_t* d_dec_in, uint8_t* d_dec_out, uint64_t dec_first_offset,
                             uint64_t dec_stride, uint64_t dec_npayloads, uint32_t dec_payload_bytes, uint32_t dec_key,
                             void* stream);

/* Duplex of two ragged relay streams (device offset / size lists, as
 * cyaes_gpu_{en,de}crypt_ragged): the stream a relay end sends and the one it
 * receives.  Same results as
 *   cyaes_gpu_encrypt_ragged(enc stream, key row enc_key)
 *   cyaes_gpu_decrypt_ragged(dec stream, key row dec_key)
 * in that order (no key arrays, no IV arrays), provided no byte of one
 * stream's payloads is a byte of the other's.  A sent stream of few, long
 * payloads (fewer than 131,072: 0xFF00-B chunks, whose CBC chains bound the
 * encrypt by their latency) is encrypted on few CUs while the received one is
 * decrypted on the others, concurrently (the decrypt on a second stream of the
 * context, joined back into `stream`); other shapes run as the two calls.
 * Meant for two streams of comparable bytes: the CU split follows the sent
 * stream's chain count, so a received stream far smaller than the sent one
 * leaves the encrypt on fewer CUs than it would take alone (~9 % longer).
 * Errors as the ragged entry points; CYAES_ERANGE for a key row >= the number
 * of keys set. */
int cyaes_gpu_duplex_ragged(cyaes_gpu* ctx, const uint8_t* d_enc_in, uint8_t* d_enc_out, const uint64_t* d_enc_offsets,
                            const uint32_t* d_enc_nbytes, uint64_t enc_npayloads, uint32_t enc_key,
                            const uint8_t* d_dec_in, uint8_t* d_dec_out, const uint64_t* d_dec_offsets,
                            const uint32_t* d_dec_nbytes, uint64_t dec_npayloads, uint32_t dec_key, void* stream);

/* ---- Host-resident uniform batches (PCIe-inclusive) ----------------------
 * The relay path starts and ends in host memory (socket buffers).  These
 * process npayloads uniform payloads that live in HOST memory: chunks of
 * chunk_bytes (0 = 256 MiB; rounded to whole payloads, and to whole sessions
 * when payloads_per_key != 0) are copied H2D, en/decrypted and copied D2H on
 * three streams (upload, compute, download) over a ring of three device slot
 * pairs, so both copy directions and the kernels overlap.  h_in / h_out may be
 * pinned (hipHostMalloc, hipHostRegister) or pageable; pageable ranges are
 * registered for the duration of the call.  h_in == h_out is allowed.  Every
 * payload is a chain from DefaultIV; key of payload p = payloads_per_key ?
 * p / payloads_per_key : 0.  Synchronous: returns when h_out is complete. */
int cyaes_gpu_encrypt_host(cyaes_gpu* ctx, const uint8_t* h_in, uint8_t* h_out, uint64_t npayloads,
                           uint32_t payload_bytes, uint32_t payloads_per_key, uint64_t chunk_bytes);
int cyaes_gpu_decrypt_host(cyaes_gpu* ctx, const uint8_t* h_in, uint8_t* h_out, uint64_t npayloads,
                           uint32_t payload_bytes, uint32_t payloads_per_key, uint64_t chunk_bytes);

/* Synchronises the device (every stream the context's batches ran on) and
 * returns CYAES_EDEVICE on an asynchronous HIP error, CYAES_ERANGE if a batch
 * since the previous check saw an out-of-range key index (the sticky flag is
 * then cleared), else CYAES_OK.  Cost: hipDeviceSynchronize, so the call
 * waits for ALL work on the device (other libraries' streams, RCCL, a running
 * batcher pipeline) and may report a fault another user of the device caused;
 * that is what charges an asynchronous fault to the check after it.  Hot
 * paths that check after each batch use cyaes_gpu_check_stream. */
int cyaes_gpu_check(cyaes_gpu* ctx);

/* The stream-scoped check: waits for `stream` only (NULL: the null stream),
 * then reads and clears the context's out-of-range flag as cyaes_gpu_check
 * does.  The flag is per context, so an ERANGE may come from a batch of this
 * context on another stream that has already finished. */
int cyaes_gpu_check_stream(cyaes_gpu* ctx, void* stream);

/* ---- Workload utilities (bench / verification; not on the hot path) ----- */
/* Synthetic plaintext of SURVEY.md §8(d): 64-bit word w of payload p is
 * splitmix64(seed + ((p0 + p) << 20) + w), little-endian. payload_bytes % 8 == 0. */
int cyaes_gpu_fill_synthetic(uint8_t* d_buf, uint64_t p0, uint64_t npayloads, uint32_t payload_bytes,
                             uint64_t seed, void* stream);
/* 128-bit order-sensitive digest of nbytes (multiple of 8):
 *   out[0] = XOR_i h_i,  out[1] = SUM_i h_i (mod 2^64),
 *   h_i = splitmix64(word_i ^ splitmix64(i)), word_i = i-th LE 64-bit word.
 * Synchronous (waits on `stream`). */
int cyaes_gpu_digest(const uint8_t* d_buf, uint64_t nbytes, uint64_t out[2], void* stream);

/* ---- Diagnostics --------------------------------------------------------
 * Host-memory registrations the library holds (cyclone_amd/csrc/cyaes_pins.cpp:
 * the batcher's packet pools and the host batches' pageable buffers; every
 * hipHostRegister the library makes goes through one process-wide registry).
 * out[0] live registrations, out[1] live registered bytes, out[2] registrations
 * made, out[3] unregistered, out[4] unregisters that failed, out[5] unregisters
 * after which the runtime still answered for the range, out[6] requests not
 * registered because another owner's registration (or a host batch's) held
 * some of their pages (pools refused, host batches bounced), out[7] references
 * held.  Out[4] and out[5] are 0 unless the runtime misbehaves; out[0] is 0
 * whenever no pool is registered and no host batch runs. */
int cyaes_debug_pins(uint64_t out[8]);
/* The host byte ranges the library has unregistered, most recent first (up to
 * the last 1,024): writes min(cap, kept) [lo, hi) pairs to out and returns
 * their number.  *outlived (nullable) = unregisters that found a page of the
 * range already unmapped, i.e. a registration that outlived its memory (the
 * precondition of a stale registration record; 0 unless a caller freed a pool
 * before unregistering it). */
uint64_t cyaes_debug_pin_history(uint64_t* out, uint64_t cap, uint64_t* outlived);

/* A context's bookkeeping: out[0] streams with a batch that read the key table
 * still in flight (entries whose batches completed are dropped on the next
 * batch or key write, so this stays bounded by the streams in use), out[1]
 * cached scratch blocks, out[2] their bytes, out[3] outgrown key tables kept
 * until destroy. */
int cyaes_debug_ctx(cyaes_gpu* ctx, uint64_t out[4]);

#ifdef __cplusplus
}
#endif

#endif /* CYAES_H */
