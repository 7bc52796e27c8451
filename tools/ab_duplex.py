#!/usr/bin/env python3
"""tools/ab_duplex.py -- interleaved A/B, in one process, of a stream of passes
run as separate encrypt and decrypt launches against the same passes run as
duplex launches (cyaes_gpu_duplex_uniform: launch k encrypts pass k while it
decrypts pass k-1; one extra launch at each end).

usage: python tools/ab_duplex.py [--payloads N] [--payload-bytes B] [--passes P] [--rounds R]
       [--lib path.so[:ENV=V...]]   (default: the product library)

Per round and mode: P passes of one batch shape (the plaintext is the same
every pass, as bench.py's passes are once filled); prints per-pass ms
(median / min over rounds) for each mode and checks both modes' ciphertext and
round-trip digests agree and restore the plaintext."""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--payloads", type=int, default=262144)
    ap.add_argument("--payload-bytes", type=int, default=65536)
    ap.add_argument("--passes", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--lib", default=None)
    args = ap.parse_args()
    import torch
    import cyclone_amd as ca

    lib = None
    if args.lib:
        path, *envs = args.lib.split(":")
        for kv in envs:
            k, v = kv.split("=", 1)
            os.environ[k] = v
        lib = ca.load_library(os.path.abspath(path))
    c = ca.GpuContext(0, lib=lib)
    c.set_keys(bytes(range(16)))
    n, pb, P = args.payloads, args.payload_bytes, args.passes
    nb = n * pb
    pt = torch.empty(nb, dtype=torch.uint8, device="cuda")
    ct = [torch.empty_like(pt), torch.empty_like(pt)]
    rt = torch.empty_like(pt)
    c.fill_synthetic(pt, 0, n, pb, 0x5EEDC1C1)
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    want_pt = c.digest(pt, nb)

    def sequential():
        for _ in range(P):
            c.encrypt_uniform(pt, ct[0], n, pb, stream=sh)
            c.decrypt_uniform(ct[0], rt, n, pb, stream=sh)

    def duplex():
        c.encrypt_uniform(pt, ct[0], n, pb, stream=sh)
        for i in range(1, P):
            c.duplex_uniform(pt, ct[i % 2], n, pb, ct[(i - 1) % 2], rt, n, pb, stream=sh)
        c.decrypt_uniform(ct[(P - 1) % 2], rt, n, pb, stream=sh)

    modes = {"sequential": sequential, "duplex": duplex}
    times = {m: [] for m in modes}
    digests = {}
    for r in range(args.rounds + 1):
        for m, fn in modes.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(s)
            fn()
            e1.record(s)
            torch.cuda.synchronize()
            if r == 0:
                digests[m] = (c.digest(ct[(P - 1) % 2 if m == "duplex" else 0], nb), c.digest(rt, nb))
                continue
            times[m].append(e0.elapsed_time(e1) / P)
    ok = digests["sequential"] == digests["duplex"] and digests["duplex"][1] == want_pt
    gib = 2.0 * nb / 2**30
    print("%d x %d B, %d passes per round, %d rounds: %s" % (n, pb, P, args.rounds,
                                                            "same-output, round trip ok" if ok else "OUTPUT DIFFERS"))
    for m in modes:
        med, mn = statistics.median(times[m]), min(times[m])
        print("  %-10s %.3f ms per pass (min %.3f)  %.1f GiB/s enc+dec" % (m, med, mn, gib / (med / 1e3)))
    print("  duplex / sequential: %.4f" % (statistics.median(times["duplex"]) / statistics.median(times["sequential"])))
    c.check()
    c.close()


if __name__ == "__main__":
    main()
