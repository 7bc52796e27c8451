#!/usr/bin/env python3
"""bench_e2e.py -- host-to-host AES-128-CBC throughput (PCIe-inclusive).

The relay path starts and ends in host memory (socket buffers, SURVEY.md
§3.1-3.2).  This measures cyaes_gpu_{en,de}crypt_host (include/cyaes.h): the
batch lives in host memory; the library streams chunks H2D -> kernel -> D2H
on three streams (upload / compute / download) over a ring of device slots,
so both copy directions overlap each other and the kernels.  Host buffers are
pinned (`--host pinned`, hipHostMalloc via torch) or pageable (`--host
pageable`, numpy; the library registers them for the call).  Reported per
direction and as the encrypt+decrypt figure of the headline metric,
2N / (t_enc + t_dec).  Not the bench.py value.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def measure(ctx, h_pt, h_ct, h_rt, n, pb, chunk, reps):
    """Best-of-`reps` seconds of cyaes_gpu_encrypt_host (h_pt -> h_ct) and
    cyaes_gpu_decrypt_host (h_ct -> h_rt) over n payloads of pb bytes in host
    memory, after one untimed encrypt that sizes the device slot ring; and
    whether the round trip restored the plaintext.  Shared with bench.py's `e2e`
    object."""
    import torch

    def run(fn, src, dst):
        t0 = time.perf_counter()
        fn(src.data_ptr(), dst.data_ptr(), n, pb, chunk_bytes=chunk)
        return time.perf_counter() - t0

    run(ctx.encrypt_host, h_pt, h_ct)  # first call sizes the device slot ring
    best_e = best_d = 1e30
    for _ in range(reps):
        best_e = min(best_e, run(ctx.encrypt_host, h_pt, h_ct))
        best_d = min(best_d, run(ctx.decrypt_host, h_ct, h_rt))
    return best_e, best_d, bool(torch.equal(h_rt, h_pt))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--payloads", type=int, default=131072)
    ap.add_argument("--payload-bytes", type=int, default=65536)
    ap.add_argument("--chunk-mib", type=int, default=256)
    ap.add_argument("--host", default="pinned", choices=["pinned", "pageable"])
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()

    import numpy as np
    import torch

    import cyclone_amd as ca

    pb, n = args.payload_bytes, args.payloads
    nbytes = n * pb
    chunk = args.chunk_mib << 20
    ctx = ca.GpuContext(0)
    ctx.set_keys(bytes(range(16)))
    pinned = args.host == "pinned"

    def hbuf():
        return torch.empty(nbytes, dtype=torch.uint8, pin_memory=pinned)
    h_pt, h_ct, h_rt = hbuf(), hbuf(), hbuf()
    # synthetic plaintext, generated on the device piece by piece
    per = max(1, (1 << 30) // pb)
    d_tmp = torch.empty(min(n, per) * pb, dtype=torch.uint8, device="cuda")
    for c0 in range(0, n, per):
        cn = min(per, n - c0)
        ctx.fill_synthetic(d_tmp, c0, cn, pb, 0x5EEDC1C1)
        h_pt[c0 * pb:(c0 + cn) * pb].copy_(d_tmp[:cn * pb])
    torch.cuda.synchronize()
    del d_tmp

    best_e, best_d, ok = measure(ctx, h_pt, h_ct, h_rt, n, pb, chunk, args.reps)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    sample = min(n, 64)
    want = oracle.batch(False, [bytes(range(16))], 0, h_pt[:sample * pb].numpy(), pb, nthreads=8)
    ok = ok and bool(np.array_equal(h_ct[:sample * pb].numpy(), want))
    gib = float(1 << 30)
    print(json.dumps({
        "metric": "AES-128-CBC host-to-host GiB/s, cyaes_gpu_{en,de}crypt_host (PCIe-inclusive)",
        "payloads": n, "payload_bytes": pb, "chunk_mib": args.chunk_mib, "host_memory": args.host,
        "encrypt_gibs": round(nbytes / best_e / gib, 2), "decrypt_gibs": round(nbytes / best_d / gib, 2),
        "enc_plus_dec_gibs": round(2 * nbytes / (best_e + best_d) / gib, 2),
        "h2d_plus_d2h_bytes_per_direction": 2 * nbytes, "parity": "bit-exact" if ok else "MISMATCH",
    }), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
