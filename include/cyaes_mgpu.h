/*
 * cyaes_mgpu.h -- single-process multi-GPU front end.
 * Library: libcyaes_mgpu.so (links libcyaes.so and RCCL).
 *
 * For a C++ host such as the relay, which runs in one process: one
 * cyaes_gpu context per device plus an RCCL communicator clique
 * (ncclCommInitAll) that carries the session keys from the owning GPU to
 * every other GPU over xGMI (ncclBroadcast), where each GPU expands them
 * itself.  Payloads are independent CBC chains (relay_local.cpp:206,
 * relay_server.cpp:472 pass no IV), so batches shard across devices with no
 * data-path collective: every device processes its own shard in its own HBM.
 * (Python / torchrun users: one process per GPU, cyclone_amd/dist.py.)
 */
#ifndef CYAES_MGPU_H
#define CYAES_MGPU_H

#include <stdint.h>

#include "cyaes.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cyaes_mgpu cyaes_mgpu;

/* devices == NULL => 0 .. ndev-1.  Creates the contexts and the RCCL clique. */
int cyaes_mgpu_create(int ndev, const int* devices, cyaes_mgpu** out);
/* Frees every device context; returns the first device's pending-fault status
 * (cyaes_gpu_destroy), else CYAES_OK. */
int cyaes_mgpu_destroy(cyaes_mgpu* mg);
int cyaes_mgpu_ndev(const cyaes_mgpu* mg);
/* The per-device context (for any cyaes_gpu_* call), or NULL. */
cyaes_gpu* cyaes_mgpu_context(cyaes_mgpu* mg, int i);

/* Copies nkeys raw 16-byte keys to device `root`, ncclBroadcast's them to all
 * devices and expands them there into each context's key table (replacing
 * it).  Synchronous. */
int cyaes_mgpu_broadcast_keys(cyaes_mgpu* mg, const uint8_t* keys, uint32_t nkeys, int root);

/* Contiguous shard of `total` payloads for device i of ndev, with boundaries
 * on multiples of `align` (use payloads_per_key so a shard starts a session). */
int cyaes_mgpu_shard(uint64_t total, int ndev, int i, uint64_t align, uint64_t* first, uint64_t* count);

/* Sharded uniform batch: device i processes npayloads[i] payloads of
 * payload_bytes in its own buffers d_in[i] -> d_out[i]; they are payloads
 * first_payload[i] ... of the global batch, so with payloads_per_key != 0
 * payload p uses key (first_payload[i] + p) / payloads_per_key of the
 * broadcast table (first_payload[i] must then be a multiple of
 * payloads_per_key).  Launches on every device, then waits for all; returns
 * the first error.  Chains start at DefaultIV (relay semantics). */
int cyaes_mgpu_encrypt_uniform(cyaes_mgpu* mg, const uint8_t* const* d_in, uint8_t* const* d_out,
                               const uint64_t* npayloads, const uint64_t* first_payload, uint32_t payload_bytes,
                               uint32_t payloads_per_key);
int cyaes_mgpu_decrypt_uniform(cyaes_mgpu* mg, const uint8_t* const* d_in, uint8_t* const* d_out,
                               const uint64_t* npayloads, const uint64_t* first_payload, uint32_t payload_bytes,
                               uint32_t payloads_per_key);

#ifdef __cplusplus
}
#endif

#endif /* CYAES_MGPU_H */
