#!/usr/bin/env python3
"""bench_e2e.py -- host-to-host AES-128-CBC throughput (PCIe-inclusive).

The relay path starts and ends in host memory (socket buffers, SURVEY.md
§3.1-3.2).  This measures the rate including hipMemcpyAsync over pinned
staging buffers: the batch lives in pinned host memory; chunks of
`--chunk-mib` are copied H2D, encrypted (or decrypted) on the GPU and copied
back D2H, with `--streams` streams in flight so copies in both directions
overlap the kernels.  Reported per direction and as the encrypt+decrypt
figure of the headline metric, 2N / (t_enc + t_dec).  Not the bench.py value.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--payloads", type=int, default=65536)
    ap.add_argument("--payload-bytes", type=int, default=65536)
    ap.add_argument("--chunk-mib", type=int, default=256)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()

    import numpy as np
    import torch

    import cyclone_amd as ca

    pb, n = args.payload_bytes, args.payloads
    nbytes = n * pb
    per_chunk = max(1, (args.chunk_mib << 20) // pb)
    chunk = per_chunk * pb
    ctx = ca.GpuContext(0)
    ctx.set_keys(bytes(range(16)))
    # pinned host batch (the "socket buffers" after gather) + staging-free device ring
    h_pt = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h_ct = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h_rt = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d_tmp = torch.empty(nbytes if nbytes < chunk else chunk, dtype=torch.uint8, device="cuda")
    ctx.fill_synthetic(d_tmp, 0, min(n, per_chunk), pb, 0x5EEDC1C1)
    for c0 in range(0, n, per_chunk):  # synthetic plaintext, generated on device chunk by chunk
        cn = min(per_chunk, n - c0)
        ctx.fill_synthetic(d_tmp, c0, cn, pb, 0x5EEDC1C1)
        h_pt[c0 * pb:(c0 + cn) * pb].copy_(d_tmp[:cn * pb])
    torch.cuda.synchronize()
    del d_tmp
    streams = [torch.cuda.Stream() for _ in range(args.streams)]
    din = [torch.empty(chunk, dtype=torch.uint8, device="cuda") for _ in streams]
    dout = [torch.empty(chunk, dtype=torch.uint8, device="cuda") for _ in streams]

    def run(decrypt, src, dst):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, c0 in enumerate(range(0, n, per_chunk)):
            k = i % len(streams)
            s = streams[k]
            cn = min(per_chunk, n - c0)
            with torch.cuda.stream(s):
                din[k][:cn * pb].copy_(src[c0 * pb:(c0 + cn) * pb], non_blocking=True)
                fn = ctx.decrypt_uniform if decrypt else ctx.encrypt_uniform
                fn(din[k], dout[k], cn, pb, stream=s.cuda_stream)
                dst[c0 * pb:(c0 + cn) * pb].copy_(dout[k][:cn * pb], non_blocking=True)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    best_e = best_d = 1e30
    for _ in range(args.reps):
        best_e = min(best_e, run(False, h_pt, h_ct))
        best_d = min(best_d, run(True, h_ct, h_rt))
    ok = bool(torch.equal(h_rt, h_pt))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    sample = min(n, 64)
    want = oracle.batch(False, [bytes(range(16))], 0, h_pt[:sample * pb].numpy(), pb, nthreads=8)
    ok = ok and bool(np.array_equal(h_ct[:sample * pb].numpy(), want))
    gib = float(1 << 30)
    print(json.dumps({
        "metric": "AES-128-CBC host-to-host GiB/s over pinned staging (PCIe-inclusive)",
        "payloads": n, "payload_bytes": pb, "chunk_mib": chunk >> 20, "streams": args.streams,
        "encrypt_gibs": round(nbytes / best_e / gib, 2), "decrypt_gibs": round(nbytes / best_d / gib, 2),
        "enc_plus_dec_gibs": round(2 * nbytes / (best_e + best_d) / gib, 2),
        "h2d_plus_d2h_bytes_per_direction": 2 * nbytes, "parity": "bit-exact" if ok else "MISMATCH",
    }), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
