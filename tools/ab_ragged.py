#!/usr/bin/env python3
"""tools/ab_ragged.py -- ragged vs uniform batch kernels on the same payloads.

Relay traffic in HBM is ragged (cyaes_relay.h: packets with 12-B headers);
this times cyaes_gpu_{en,de}crypt_ragged on N equal payloads laid out
contiguously (offsets = p * size) against the uniform entry points, and on a
relay-packet stream layout (payload at packet offset 12, 4-B aligned).
usage: python tools/ab_ragged.py [--rounds 5] [--lib build/variants/x.so]"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--lib", default=None, help="a variant libcyaes.so (make variant)")
    ap.add_argument("--sizes", default=None, help="n:pb,... (default: the four below)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import cyclone_amd as ca
    c = ca.GpuContext(0, lib=ca.load_library(os.path.abspath(args.lib)) if args.lib else None)
    c.set_keys(bytes(range(16)))
    s = torch.cuda.current_stream()
    sizes = ((21000, 1472), (262144, 1472), (1048576, 1472), (65536, 65280))
    if args.sizes:
        sizes = tuple(tuple(int(v) for v in x.split(":")) for x in args.sizes.split(","))
    for n, pb in sizes:
        nbytes = n * pb
        pt = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        c.fill_synthetic(pt, 0, n, pb, 0x5EEDC1C1)
        ct_u, ct_r, rt_u, rt_r = (torch.empty_like(pt) for _ in range(4))
        off = torch.from_numpy(np.arange(n, dtype=np.uint64) * pb).to("cuda")
        nb = torch.full((n,), pb, dtype=torch.int32, device="cuda")
        # relay stream: packet = 4-B head + 8-B forward msg + payload, back to back
        pk = pb + 12
        srel = torch.zeros(n * pk, dtype=torch.uint8, device="cuda")
        srel.view(n, pk)[:, 12:] = pt.view(n, pb)
        off_rel = torch.from_numpy(np.arange(n, dtype=np.uint64) * pk + 12).to("cuda")
        t = {k: [] for k in ("enc_uniform", "enc_ragged", "enc_relay", "dec_uniform", "dec_ragged", "dec_relay")}
        for r in range(args.rounds + 1):
            runs = [("enc_uniform", lambda: c.encrypt_uniform(pt, ct_u, n, pb, stream=s.cuda_stream)),
                    ("enc_ragged", lambda: c.encrypt_ragged(pt, ct_r, off, nb, n, stream=s.cuda_stream)),
                    ("enc_relay", lambda: c.encrypt_ragged(srel, srel, off_rel, nb, n, stream=s.cuda_stream)),
                    ("dec_uniform", lambda: c.decrypt_uniform(ct_u, rt_u, n, pb, stream=s.cuda_stream)),
                    ("dec_ragged", lambda: c.decrypt_ragged(ct_u, rt_r, off, nb, n, stream=s.cuda_stream)),
                    ("dec_relay", lambda: c.decrypt_ragged(srel, srel, off_rel, nb, n, stream=s.cuda_stream))]
            for k, f in runs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                f()
                e1.record(s)
                torch.cuda.synchronize()
                if r:
                    t[k].append(e0.elapsed_time(e1))
        ok = torch.equal(ct_u, ct_r) and torch.equal(rt_u, pt) and torch.equal(rt_r, pt) and \
            torch.equal(srel.view(n, pk)[:, 12:].reshape(-1), pt)  # relay stream: enc then dec in place, round trip
        print("%8d x %6d B: " % (n, pb) + "  ".join("%s %.4f" % (k, statistics.median(v)) for k, v in t.items()) +
              " ms  " + ("ok" if ok else "MISMATCH"), flush=True)
        del pt, ct_u, ct_r, rt_u, rt_r, srel
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
