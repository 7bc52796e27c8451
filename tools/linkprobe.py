#!/usr/bin/env python3
"""linkprobe.py -- host<->device copy ceilings for the end-to-end path.

Measures pinned H2D alone, D2H alone and both directions at once (two
streams), the ceiling bench_e2e.py's H2D -> kernel -> D2H pipeline can reach.
Prints one JSON line (GB/s = 1e9 B/s and GiB/s).
"""
import argparse
import json
import time


def measure(torch, nbytes, chunk, reps=3):
    """Pinned host<->device copy ceilings: best-of-`reps` H2D alone, D2H alone
    and both at once on two streams, `nbytes` per direction in `chunk`-byte
    copies.  Returns the JSON-able dict (GB/s = 1e9 B/s).  Shared with
    bench.py's `e2e` object."""
    n, c = nbytes, chunk
    h_src = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h_dst = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h_src.fill_(7)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    s_up, s_dn = torch.cuda.Stream(), torch.cuda.Stream()

    def h2d():
        with torch.cuda.stream(s_up):
            for o in range(0, n, c):
                d[o:o + c].copy_(h_src[o:o + c], non_blocking=True)

    def d2h():
        with torch.cuda.stream(s_dn):
            for o in range(0, n, c):
                h_dst[o:o + c].copy_(d2[o:o + c], non_blocking=True)

    def timed(fns):
        best = 1e30
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for f in fns:
                f()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    t_up = timed([h2d])
    t_dn = timed([d2h])
    t_both = timed([h2d, d2h])
    del h_src, h_dst, d, d2
    return {"bytes_per_direction": n, "chunk_mib": c >> 20,
            "h2d_gbs": round(n / t_up / 1e9, 2), "d2h_gbs": round(n / t_dn / 1e9, 2),
            "duplex_gbs_per_direction": round(n / t_both / 1e9, 2),
            "duplex_gibs_per_direction": round(n / t_both / 2**30, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=4096, help="bytes moved per direction")
    ap.add_argument("--chunk-mib", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    print(json.dumps(measure(torch, a.mib << 20, a.chunk_mib << 20, a.reps)), flush=True)


if __name__ == "__main__":
    main()
