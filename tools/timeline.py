#!/usr/bin/env python3
"""tools/timeline.py -- where a launch's time goes, wave by wave.

Runs one encrypt and one decrypt launch of a config on the clock-probe build
(build/variants/clockprobe.so, CYAES_CLOCK_PROBE: every wave records its start
and end on the 100 MHz s_memrealtime clock, its shader cycles, HW_ID and
XCC_ID) after a warm-up, and prints per launch: the span, the spread of wave
start and end times, per-XCD means and clocks, the spread of per-CU finish
times, and the spread inside workgroups.  The question it answers: is a
launch's tail the waves of a few slow CUs / XCDs (a dynamic work split helps)
or uniform (it does not).

usage: python tools/timeline.py [--config B|C|D|relay|relay_strided] [--lib build/variants/clockprobe.so]
       [--reps 3] [--duplex] [ENV=VALUE ...]   (context settings, e.g. CYAES_DEC_DYN=0)
--duplex: one duplex launch (cyaes_gpu_duplex_uniform: the config's encrypt and,
in the same grid, the decrypt of its ciphertext) instead of the two launches;
its encrypt and decrypt phases are reported on one clock (the launch's first
wave start).
"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
WAVES = 8192


def records(lib, kind, tus=(0, 1, 2, 4)):
    """Timeline records of the last launch of `kind` (0 enc, 1 dec) from whichever kernel TU ran it."""
    out = []
    for tu in tus:
        buf = (ctypes.c_uint32 * (8 * WAVES))()
        if lib.cyaes_debug_timeline(tu, kind, buf) != 0:
            raise SystemExit("cyaes_debug_timeline failed (not a clock-probe build?)")
        for w in range(WAVES):
            r = buf[8 * w: 8 * w + 8]
            if r[1] == 0 and r[0] == 0:
                continue
            out.append({"start": r[0], "end": r[1], "hw": r[2], "xcc": r[3] & 0xF,
                        "cycles": r[4] | (r[5] << 32), "block": r[6], "wave": r[7], "tu": tu})
    return out


def report(name, recs, t0=None):
    if not recs:
        print("%s: no records" % name)
        return
    if t0 is None:
        t0 = min(r["start"] for r in recs)
    for r in recs:  # 32-bit tick counters: relative to the launch's first start (wraps every 42 s)
        r["s"] = ((r["start"] - t0) & 0xFFFFFFFF) / 1e5  # ms
        r["e"] = ((r["end"] - t0) & 0xFFFFFFFF) / 1e5
        r["cu"] = (r["xcc"], (r["hw"] >> 13) & 7, (r["hw"] >> 12) & 1, (r["hw"] >> 8) & 15)
    ends = sorted(r["e"] for r in recs)
    starts = sorted(r["s"] for r in recs)
    q = lambda v, f: v[min(len(v) - 1, int(f * len(v)))]
    span = ends[-1]
    ticks = sum((r["end"] - r["start"]) & 0xFFFFFFFF for r in recs)
    print("%s: %d waves (TU %s), span %.3f ms, clock %.3f GHz" % (
        name, len(recs), sorted({r["tu"] for r in recs}), span, sum(r["cycles"] for r in recs) / ticks * 0.1))
    print("  wave start: max %.3f ms | wave end: mean %.3f p10 %.3f p50 %.3f p90 %.3f p99 %.3f max %.3f ms "
          "(max/mean %.3f)" % (starts[-1], statistics.mean(ends), q(ends, .1), q(ends, .5), q(ends, .9),
                               q(ends, .99), ends[-1], ends[-1] / statistics.mean(ends)))
    xccs = sorted({r["xcc"] for r in recs})
    for x in xccs:
        rs = [r for r in recs if r["xcc"] == x]
        tk = sum((r["end"] - r["start"]) & 0xFFFFFFFF for r in rs)
        print("  XCD %d: %4d waves, end mean %.3f max %.3f ms, clock %.3f GHz" % (
            x, len(rs), statistics.mean(r["e"] for r in rs), max(r["e"] for r in rs),
            sum(r["cycles"] for r in rs) / tk * 0.1))
    cus = {}
    for r in recs:
        cus.setdefault(r["cu"], []).append(r["e"])
    cmax = sorted(max(v) for v in cus.values())
    cmean = sorted(statistics.mean(v) for v in cus.values())
    print("  per CU (%d): finish (last wave) min %.3f p50 %.3f max %.3f ms; mean wave end min %.3f max %.3f ms" % (
        len(cus), cmax[0], q(cmax, .5), cmax[-1], cmean[0], cmean[-1]))
    blocks = {}
    for r in recs:
        blocks.setdefault(r["block"], []).append(r["e"])
    spread = [max(v) - min(v) for v in blocks.values() if len(v) > 1]
    if spread:
        print("  inside a workgroup: last - first wave end mean %.3f max %.3f ms" % (statistics.mean(spread),
                                                                                   max(spread)))
    slow = sorted(recs, key=lambda r: -r["e"])[:5]
    print("  slowest waves: " + ", ".join("xcd %d cu %s blk %d w %d end %.3f" % (
        r["xcc"], r["cu"][1:], r["block"], r["wave"], r["e"]) for r in slow))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="B", choices=["B", "C", "D", "relay", "relay_strided"])
    ap.add_argument("--lib", default=os.path.join(ROOT, "build", "variants", "clockprobe.so"))
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--duplex", action="store_true")
    ap.add_argument("env", nargs="*")
    args = ap.parse_args()
    for kv in args.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    import torch
    import bench
    import cyclone_amd as ca
    lib = ca.load_library(os.path.abspath(args.lib))
    lib.cyaes_debug_timeline.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    c = ca.GpuContext(0, lib=lib)
    n, pb, ppk = {"B": (1 << 20, 1472, 0), "C": (1 << 18, 65536, 0), "D": (1 << 20, 1472, 256),
                  "relay": (1 << 20, 1472, 0), "relay_strided": (1 << 20, 1472, 0)}[args.config]
    c.set_keys(bench.session_keys(n // ppk) if ppk else bytes(range(16)))
    s = torch.cuda.current_stream().cuda_stream
    pt = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
    c.fill_synthetic(pt, 0, n, pb, 0x5EEDC1C1)
    if args.config.startswith("relay"):  # relay packets in place: payload at 12 + p * 1,484
        hdr, stride = 12, pb + 12
        buf = torch.full((n * stride + 16,), 0xA5, dtype=torch.uint8, device="cuda")
        buf[: n * stride].view(n, stride)[:, hdr:hdr + pb] = pt.view(n, pb)
    if args.config == "relay_strided":
        enc = lambda: c.encrypt_strided(buf, buf, hdr, stride, n, pb, stream=s)
        dec = lambda: c.decrypt_strided(buf, buf, hdr, stride, n, pb, stream=s)
    elif args.config == "relay":
        off = torch.arange(n, dtype=torch.int64, device="cuda") * stride + hdr
        nb = torch.full((n,), pb, dtype=torch.int32, device="cuda")
        enc = lambda: c.encrypt_ragged(buf, buf, off, nb, n, stream=s)
        dec = lambda: c.decrypt_ragged(buf, buf, off, nb, n, stream=s)
    else:
        ct = torch.empty_like(pt)
        rt = torch.empty_like(pt)
        enc = lambda: c.encrypt_uniform(pt, ct, n, pb, payloads_per_key=ppk, stream=s)
        dec = lambda: c.decrypt_uniform(ct, rt, n, pb, payloads_per_key=ppk, stream=s)
    for _ in range(20 if pb < 65536 else 3):  # clock ramp
        enc()
        dec()
    torch.cuda.synchronize()
    if args.duplex:
        ct2 = torch.empty_like(pt)
        for rep in range(args.reps):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            c.duplex_uniform(pt, ct2, n, pb, ct, rt, n, pb, stream=s)  # encrypt pt while ct is decrypted
            ev[1].record()
            torch.cuda.synchronize()
            re_, rd = records(lib, 0, (3,)), records(lib, 1, (3,))
            t0 = min(r["start"] for r in re_)
            print("== config %s rep %d: duplex launch %.3f ms (events) %s" % (
                args.config, rep, ev[0].elapsed_time(ev[1]), " ".join(args.env)))
            report("duplex encrypt phase", re_, t0)
            report("duplex decrypt phase", rd, t0)
        assert torch.equal(rt, pt) and torch.equal(ct2, ct)
        c.close()
        return
    for rep in range(args.reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        enc()
        ev[1].record()
        torch.cuda.synchronize()
        re_ = records(lib, 0)
        ev[2].record()
        dec()
        ev[3].record()
        torch.cuda.synchronize()
        rd = records(lib, 1)
        print("== config %s rep %d: encrypt %.3f ms, decrypt %.3f ms (events) %s" % (
            args.config, rep, ev[0].elapsed_time(ev[1]), ev[2].elapsed_time(ev[3]), " ".join(args.env)))
        report("encrypt", re_)
        report("decrypt", rd)
    c.close()


if __name__ == "__main__":
    main()
