"""Multi-process (world_size 2, gloo, CPU) coverage of the N>1 path of bench.py:
key broadcast from rank 0, contiguous payload shards, per-rank keyed batches.
Every rank runs the oracle on its shard; the union must equal the
single-process result for the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cyclone_amd import dist as cdist

PB, PER_RANK, PPK = 160, 24, 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _keys(n):
    rng = np.random.default_rng(2024)
    return rng.integers(0, 256, 16 * n, dtype=np.uint8).tobytes()


def _worker(rank, world, port, outdir):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        total = PER_RANK * world
        nkeys = cdist.session_range(0, total, PPK)[1]
        keys = cdist.broadcast_keys(_keys(nkeys) if rank == 0 else None, nkeys, "cpu")
        p0, n = cdist.weak_shard(PER_RANK, rank)
        k0, nk = cdist.session_range(p0, n, PPK)
        raw = keys.numpy().tobytes()
        mine = [raw[16 * k:16 * k + 16] for k in range(k0, k0 + nk)]
        pt = oracle.synthetic(p0, n, PB)
        ct = oracle.batch(False, mine, PPK, pt, PB)
        assert np.array_equal(oracle.batch(True, mine, PPK, ct, PB), pt)
        t = torch.from_numpy(ct.copy())
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        if rank == 0:
            np.save(os.path.join(outdir, "gathered.npy"), torch.cat(parts).numpy())
            np.save(os.path.join(outdir, "keys.npy"), keys.numpy())
    finally:
        dist.destroy_process_group()


def test_shard_ranges_cover_batch():
    for total, world, align in [(1000, 8, 1), (1 << 20, 8, 256), (37, 4, 5), (3, 4, 1)]:
        ranges = [cdist.shard(total, r, world, align) for r in range(world)]
        pos = 0
        for p0, n in ranges:
            assert p0 == pos and n >= 0
            assert p0 % align == 0 or n == 0
            pos += n
        assert pos == total
    assert cdist.weak_shard(262144, 3) == (3 * 262144, 262144)
    assert cdist.session_range(512, 256, 256) == (2, 1)
    assert cdist.session_range(100, 200, 0) == (0, 1)


def test_two_ranks_match_single_process(tmp_path):
    import oracle
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    gathered = np.load(tmp_path / "gathered.npy")
    keys = np.load(tmp_path / "keys.npy").tobytes()
    total = PER_RANK * world
    nkeys = cdist.session_range(0, total, PPK)[1]
    assert keys == _keys(nkeys)  # broadcast delivered rank 0's keys
    full = oracle.batch(False, [keys[16 * k:16 * k + 16] for k in range(nkeys)], PPK,
                        oracle.synthetic(0, total, PB), PB)
    assert np.array_equal(gathered, full)
