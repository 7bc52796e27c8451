#!/usr/bin/env python3
"""tools/ab_stride.py -- ragged encrypt time against the packet stride.

N payloads of PB bytes, 16-B aligned, laid out at a fixed stride (payload p at
p * stride); out of place.  Separates the cost of the stride (line phase of
each lane's payload) from misalignment and in-place effects
(tools/ab_relay_layout.py).  usage: python tools/ab_stride.py [--strides 1472,1488,...]"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1048576)
    ap.add_argument("--pb", type=int, default=1472)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--strides", default="1472,1488,1504,1536,1600,2048,2944,1472")
    args = ap.parse_args()
    import numpy as np
    import torch
    import cyclone_amd as ca
    c = ca.GpuContext(0)
    c.set_keys(bytes(range(16)))
    s = torch.cuda.current_stream()
    n, pb = args.n, args.pb
    pt = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
    c.fill_synthetic(pt, 0, n, pb, 0x5EEDC1C1)
    ref = torch.empty_like(pt)
    c.encrypt_uniform(pt, ref, n, pb, stream=s.cuda_stream)
    nb = torch.full((n,), pb, dtype=torch.int32, device="cuda")
    for stride in (int(x) for x in args.strides.split(",")):
        src = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
        src.view(n, stride)[:, :pb] = pt.view(n, pb)
        dst = torch.zeros_like(src)
        off = torch.from_numpy(np.arange(n, dtype=np.uint64) * stride).to("cuda")
        ts = []
        for r in range(args.rounds + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            c.encrypt_ragged(src, dst, off, nb, n, stream=s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
        ok = torch.equal(dst.view(n, stride)[:, :pb].reshape(-1), ref)
        print("stride %5d (%% 128 = %3d): enc %.4f ms (min %.4f)  %s" %
              (stride, stride % 128, statistics.median(ts), min(ts), "ok" if ok else "MISMATCH"), flush=True)
        del src, dst
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
