"""Multi-GPU plumbing for the batched AES path.

One process per GPU (torchrun).  Payloads are independent CBC chains
(relay_local.cpp:206 / relay_server.cpp:329 pass no IV), so a batch shards
into contiguous payload ranges with no data-path collective.  The only
collective is the session-key broadcast from rank 0 (the relay's DH secret
owner, relay_server.cpp:218-240): over RCCL (backend "nccl") on MI355X it
travels over xGMI into device memory, where cyaes_gpu_set_keys_device
expands it; the same code runs on gloo for CPU tests.
"""
import torch
import torch.distributed as dist


def shard(npayloads, rank, world, align=1):
    """Contiguous payload range [p0, p0 + n) of `rank` for a fixed total (strong
    scaling).  Boundaries fall on multiples of `align` (use payloads_per_key so
    a rank's batch starts on a session boundary)."""
    if world < 1 or not 0 <= rank < world or align < 1:
        raise ValueError("bad rank/world/align")
    units = (npayloads + align - 1) // align

    def start(r):
        return min(npayloads, units * r // world * align)
    return start(rank), start(rank + 1) - start(rank)


def weak_shard(per_rank, rank):
    """Payload range of `rank` when every rank processes `per_rank` payloads (weak scaling)."""
    return per_rank * rank, per_rank


def session_range(p0, n, payloads_per_key):
    """Session keys [k0, k0 + nk) that payloads [p0, p0 + n) use (payload p -> key p // ppk)."""
    if not payloads_per_key:
        return 0, 1
    k0 = p0 // payloads_per_key
    return k0, (p0 + n - 1) // payloads_per_key - k0 + 1


def broadcast_keys(keys, nkeys, device, src=0, group=None):
    """Broadcasts nkeys raw 16-byte keys from `src`; returns a uint8 tensor of
    nkeys*16 bytes on `device` on every rank.  `keys` (bytes) is read on src only."""
    if dist.is_available() and dist.is_initialized() and dist.get_rank(group) == src or \
            not (dist.is_available() and dist.is_initialized()):
        if keys is None or len(keys) != 16 * nkeys:
            raise ValueError("src rank must supply nkeys*16 key bytes")
        t = torch.frombuffer(bytearray(keys), dtype=torch.uint8).to(device)
    else:
        t = torch.zeros(16 * nkeys, dtype=torch.uint8, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.broadcast(t, src=src, group=group)
    return t
