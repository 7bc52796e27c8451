#!/usr/bin/env python3
"""tools/ab_xcd_weights.py -- the XCD-weighted static decrypt split (VERDICT r05
next 7), calibrated and A/B'd on the box it runs on, in ONE process.

1. Calibrate: on the clock-probe build (build/variants/clockprobe.so), decrypt
   config B / D with the default (equal) static split and record every wave's
   start and end; a slot's speed is 1 / the mean wave time of its workgroups
   (slot = workgroup index mod 8, which the dispatcher maps to XCD 0..7 in turn;
   the hardware XCC_ID is printed beside it).
2. A/B, interleaved rounds: libcyaes.so contexts with the equal split, the
   weighted split (CYAES_DEC_XCD_W = the measured speeds), the weights'
   deviation doubled, and the dynamic pool at 100 %; median / min decrypt ms,
   outputs checked against the equal split's.
3. The weighted split on the clock-probe build: did the slots' ends converge?

usage: python tools/ab_xcd_weights.py [--config B|D] [--rounds 10] [--calib 5]
"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="B", choices=["B", "D"])
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--calib", type=int, default=5)
    args = ap.parse_args()
    import torch
    import bench
    import cyclone_amd as ca
    import timeline

    n, pb, ppk = {"B": (1 << 20, 1472, 0), "D": (1 << 20, 1472, 256)}[args.config]
    keys = bench.session_keys(n // ppk) if ppk else bytes(range(16))
    s = torch.cuda.current_stream().cuda_stream
    pt = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
    ct = torch.empty_like(pt)

    def with_env(env, fn):
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            return fn()
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    plib = ca.load_library(os.path.join(ROOT, "build", "variants", "clockprobe.so"))
    plib.cyaes_debug_timeline.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]

    def probe(env, reps, label):
        c = with_env(env, lambda: ca.GpuContext(0, lib=plib))
        c.set_keys(keys)
        c.fill_synthetic(pt, 0, n, pb, bench.PLAINTEXT_SEED, s)
        c.encrypt_uniform(pt, ct, n, pb, payloads_per_key=ppk, stream=s)
        rt = torch.empty_like(pt)
        for _ in range(20):
            c.decrypt_uniform(ct, rt, n, pb, payloads_per_key=ppk, stream=s)
        torch.cuda.synchronize()
        per_slot = {x: [] for x in range(8)}
        ends = {x: [] for x in range(8)}
        hw = {x: set() for x in range(8)}
        tails = []
        for _ in range(reps):
            c.decrypt_uniform(ct, rt, n, pb, payloads_per_key=ppk, stream=s)
            torch.cuda.synchronize()
            recs = timeline.records(plib, 1)
            t0 = min(r["start"] for r in recs)
            e_all = []
            for r in recs:
                x = r["block"] % 8
                dur = ((r["end"] - r["start"]) & 0xFFFFFFFF) / 1e5
                per_slot[x].append(dur)
                e = ((r["end"] - t0) & 0xFFFFFFFF) / 1e5
                ends[x].append(e)
                e_all.append(e)
                hw[x].add(r["xcc"])
            tails.append(max(e_all) / statistics.mean(e_all))
        assert torch.equal(rt, pt)
        c.close()
        print("%s: %d launches, wave-end max/mean %.3f" % (label, reps, statistics.mean(tails)))
        for x in range(8):
            print("  slot %d (XCC %s): mean wave %.4f ms, mean end %.4f max end %.4f ms" % (
                x, sorted(hw[x]), statistics.mean(per_slot[x]), statistics.mean(ends[x]), max(ends[x])))
        return [1.0 / statistics.mean(per_slot[x]) for x in range(8)]

    speed = probe({}, args.calib, "calibration, equal split")
    mean = statistics.mean(speed)
    w = [v / mean for v in speed]
    w2 = [1 + 2 * (v - 1) for v in w]
    fmt = lambda ws: ",".join("%.4f" % v for v in ws)  # noqa: E731
    print("weights (slot speed / mean): %s" % fmt(w))
    specs = [("equal", {}), ("weighted", {"CYAES_DEC_XCD_W": fmt(w)}),
             ("weighted x2", {"CYAES_DEC_XCD_W": fmt(w2)}),
             ("pool 100 %", {"CYAES_DEC_DYN": "1", "CYAES_DEC_DYN_PCT": "100"})]
    ctxs = []
    for name, env in specs:
        c = with_env(env, lambda: ca.GpuContext(0))
        c.set_keys(keys)
        ctxs.append((name, c, torch.empty_like(pt)))
    ctxs[0][1].fill_synthetic(pt, 0, n, pb, bench.PLAINTEXT_SEED, s)
    ctxs[0][1].encrypt_uniform(pt, ct, n, pb, payloads_per_key=ppk, stream=s)
    res = {name: [] for name, _, _ in ctxs}
    for r in range(args.rounds + 1):
        order = ctxs if r % 2 == 0 else ctxs[::-1]
        for name, c, rt in order:
            evs = []
            for k in range(6):  # steady state: back to back, the last 3 timed
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                c.decrypt_uniform(ct, rt, n, pb, payloads_per_key=ppk, stream=s)
                b.record()
                if k >= 3:
                    evs.append((a, b))
            torch.cuda.synchronize()
            if r:
                res[name] += [a.elapsed_time(b) for a, b in evs]
    for name, c, rt in ctxs:
        assert torch.equal(rt, pt), name
        print("%-14s decrypt med %.4f min %.4f ms (%d launches) same-output" % (
            name, statistics.median(res[name]), min(res[name]), len(res[name])))
        c.close()
    probe({"CYAES_DEC_XCD_W": fmt(w)}, args.calib, "weighted split on the clock-probe build")


if __name__ == "__main__":
    main()
