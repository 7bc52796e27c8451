#!/usr/bin/env python3
"""tools/ab_quad.py -- encrypt time of one lane per chain (k_encrypt) vs four
lanes per chain (k_encrypt_quad) over batch sizes, interleaved in one process.

Contexts are created with CYAES_QUAD_MAX_CHAINS = 0 (lane kernel always),
the library default, and 2^40 (quad kernel always); outputs must agree.
usage: python tools/ab_quad.py [--rounds 5]"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIZES = [(1, 1472), (64, 1472), (4096, 1024), (16384, 1472), (65535, 1472), (131072, 1472), (262144, 1472),
         (1048576, 1472), (16384, 65536), (65535, 65536), (131072, 65536)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import torch
    import cyclone_amd as ca
    ctxs = {}
    for name, v in (("lane", "0"), ("default", None), ("quad", str(1 << 40))):
        if v is None:
            os.environ.pop("CYAES_QUAD_MAX_CHAINS", None)
        else:
            os.environ["CYAES_QUAD_MAX_CHAINS"] = v
        c = ca.GpuContext(0)
        c.set_keys(bytes(range(16)))
        ctxs[name] = c
    os.environ.pop("CYAES_QUAD_MAX_CHAINS", None)
    s = torch.cuda.current_stream()
    for n, pb in SIZES:
        nbytes = n * pb
        pt = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        ctxs["lane"].fill_synthetic(pt, 0, n, pb, 0x5EEDC1C1)
        outs = {k: torch.empty_like(pt) for k in ctxs}
        t = {k: [] for k in ctxs}
        for r in range(args.rounds + 1):
            for k, c in ctxs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                c.encrypt_uniform(pt, outs[k], n, pb, stream=s.cuda_stream)
                e1.record(s)
                torch.cuda.synchronize()
                if r:
                    t[k].append(e0.elapsed_time(e1))
        same = all(torch.equal(outs["lane"], o) for o in outs.values())
        med = {k: statistics.median(v) for k, v in t.items()}
        print("%8d x %6d B: " % (n, pb) + "  ".join("%s %.4f ms" % (k, med[k]) for k in ctxs) +
              "  lane/quad %.2fx  %s" % (med["lane"] / med["quad"], "same-output" if same else "MISMATCH"), flush=True)
        del pt, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
