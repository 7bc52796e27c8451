#!/usr/bin/env python3
"""tools/ab.py -- interleaved A/B timing of libcyaes.so variants in ONE process
(MI355X_MICROARCH.md: never rank builds by timings from different runs/devices).

usage: python tools/ab.py build/variants/a.so build/variants/b.so [--rounds 6] [--payloads N]
       [--payload-bytes B] [--ppk K]   (--ppk: sessions of K payloads, config D's keys)
       [--relay]   (the payloads inside relay packets, 12-B headers, stride B + 12, ragged kernels
                    in place, as bench.py's relay_stream)
A library may carry context settings: path:NAME=VALUE[:NAME=VALUE] sets those
environment variables while its context is created (e.g. the same library
twice, once with CYAES_ENC_RUN=1).
Each round runs every variant's encrypt and decrypt once on the same config-C
buffers; prints per-variant median/min ms per kernel and checks the outputs agree.
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--payloads", type=int, default=262144)
    ap.add_argument("--payload-bytes", type=int, default=65536)
    ap.add_argument("--ppk", type=int, default=0, help="payloads per session key (0: one key)")
    ap.add_argument("--key-idx", action="store_true", help="with --ppk: the same sessions as a per-payload index array")
    ap.add_argument("--relay", action="store_true", help="relay packet stream in place (ragged kernels)")
    ap.add_argument("--flush-between", action="store_true",
                    help="overwrite a 1-GiB scratch tensor between the encrypt and the decrypt (evicts the caches; "
                         "the decrypt is timed from after it)")
    ap.add_argument("--sync-between", action="store_true",
                    help="device synchronisation between the encrypt and the decrypt launch (the decrypt starts idle)")
    ap.add_argument("--relay-api", default="ragged", choices=["ragged", "strided"],
                    help="--relay: the ragged entry points (device lists) or the strided ones")
    args = ap.parse_args()
    import torch
    import cyclone_amd as ca

    n, pb = args.payloads, args.payload_bytes
    nbytes = n * pb
    ctxs = []
    for spec in args.libs:
        path, *envs = spec.split(":")
        saved = {}
        for kv in envs:
            k, v = kv.split("=", 1)
            saved[k] = os.environ.get(k)
            os.environ[k] = v
        lib = ca.load_library(os.path.abspath(path))
        c = ca.GpuContext(0, lib=lib)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        if args.ppk:
            import bench
            c.set_keys(bench.session_keys((args.payloads + args.ppk - 1) // args.ppk))
        else:
            c.set_keys(bytes(range(16)))
        ctxs.append(c)
    pt = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    ct = torch.empty_like(pt)
    rt = torch.empty_like(pt)
    ctxs[0].fill_synthetic(pt, 0, n, pb, 0x5EEDC1C1)
    s = torch.cuda.current_stream()
    if args.relay:
        return relay(args, ctxs, pt, torch, s)
    kidx = None
    if args.key_idx and args.ppk:
        kidx = (torch.arange(n, dtype=torch.int64, device="cuda") // args.ppk).to(torch.int32)
    times = {p: {"enc": [], "dec": []} for p in args.libs}  # keyed by spec
    probes = {}
    digests = {}
    for r in range(args.rounds + 1):
        for path, c in zip(args.libs, ctxs):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(s)
            c.encrypt_uniform(pt, ct, n, pb, key_idx=kidx, payloads_per_key=0 if kidx is not None else args.ppk,
                              stream=s.cuda_stream)
            e[1].record(s)
            flush(args, torch, e, s)
            if args.sync_between:
                torch.cuda.synchronize()
            c.decrypt_uniform(ct, rt, n, pb, key_idx=kidx, payloads_per_key=0 if kidx is not None else args.ppk,
                              stream=s.cuda_stream)
            e[2].record(s)
            torch.cuda.synchronize()
            if r == 0:  # warm-up round; check outputs
                digests[path] = (c.digest(ct, nbytes), c.digest(rt, nbytes))
                probe(c, None)
                continue
            probe(c, probes.setdefault(path, []))
            times[path]["enc"].append(e[0].elapsed_time(e[1]))
            times[path]["dec"].append((e[3] if len(e) > 3 else e[1]).elapsed_time(e[2]))
    ref = digests[args.libs[0]]
    for path in args.libs:
        t = times[path]
        print("%-40s enc med %.3f min %.3f | dec med %.3f min %.3f | %s" % (
            path.replace(ROOT + "/", "").replace("cyclone_amd/", ""), statistics.median(t["enc"]), min(t["enc"]), statistics.median(t["dec"]),
            min(t["dec"]), "same-output" if digests[path] == ref else "OUTPUT DIFFERS"))
        for kind, v in zip(("enc", "dec"), zip(*probes.get(path, []))):
            cyc, tick, waves, tmax = (sum(x[i] for x in v) for i in range(4))
            if waves:
                print("    %s clock %.3f GHz, mean wave %.3f ms, max wave %.3f ms (per launch)" % (
                    kind, cyc / tick * 0.1, tick / waves / 1e5, tmax / len(v) / 1e5))


_scratch = []


def flush(args, torch, e, s):
    """--flush-between: evict the caches between the launches; the decrypt is then timed from e[3]."""
    if not args.flush_between:
        return
    if not _scratch:
        _scratch.append(torch.empty(1 << 30, dtype=torch.uint8, device="cuda"))
    _scratch[0].fill_(0x3C)
    e.append(torch.cuda.Event(enable_timing=True))
    e[-1].record(s)


def relay(args, ctxs, pt, torch, s):
    """Interleaved in-place ragged encrypt + decrypt of a relay packet stream."""
    n, pb = args.payloads, args.payload_bytes
    hdr, stride = 12, pb + 12
    buf = torch.full((n * stride + 16,), 0xA5, dtype=torch.uint8, device="cuda")
    view = buf[: n * stride].view(n, stride)
    d_off = torch.arange(n, dtype=torch.int64, device="cuda") * stride + hdr
    d_nb = torch.full((n,), pb, dtype=torch.int32, device="cuda")
    times = {p: {"enc": [], "dec": []} for p in args.libs}
    digests = {}
    for r in range(args.rounds + 1):
        for path, c in zip(args.libs, ctxs):
            view[:, hdr:hdr + pb] = pt.view(n, pb)
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(s)
            if args.relay_api == "strided":
                c.encrypt_strided(buf, buf, hdr, stride, n, pb, stream=s.cuda_stream)
            else:
                c.encrypt_ragged(buf, buf, d_off, d_nb, n, stream=s.cuda_stream)
            e[1].record(s)
            flush(args, torch, e, s)
            if r == 0 or args.sync_between:
                torch.cuda.synchronize()
            if r == 0:
                dct = c.digest(buf, n * stride)
            if args.relay_api == "strided":
                c.decrypt_strided(buf, buf, hdr, stride, n, pb, stream=s.cuda_stream)
            else:
                c.decrypt_ragged(buf, buf, d_off, d_nb, n, stream=s.cuda_stream)
            e[2].record(s)
            torch.cuda.synchronize()
            if r == 0:
                ok = bool(torch.equal(view[:, hdr:hdr + pb].reshape(-1), pt)) and bool((view[:, :hdr] == 0xA5).all())
                digests[path] = (dct, ok)
                continue
            times[path]["enc"].append(e[0].elapsed_time(e[1]))
            times[path]["dec"].append((e[3] if len(e) > 3 else e[1]).elapsed_time(e[2]))
    ref = digests[args.libs[0]][0]
    for path in args.libs:
        t = times[path]
        print("%-40s relay enc med %.3f min %.3f | dec med %.3f min %.3f | %s" % (
            path.replace(ROOT + "/", "").replace("cyclone_amd/", ""), statistics.median(t["enc"]), min(t["enc"]),
            statistics.median(t["dec"]), min(t["dec"]),
            ("same-output" if digests[path][0] == ref else "OUTPUT DIFFERS") +
            ("" if digests[path][1] else " ROUND TRIP FAILED")))


def probe(ctx, sink):
    """Reads (and clears) the CYAES_CLOCK_PROBE sums of a variant build, if it has them."""
    import ctypes
    fn = getattr(ctx._lib, "cyaes_debug_probe", None)
    if fn is None:
        return
    buf = (ctypes.c_ulonglong * 8)()
    fn(buf)
    if sink is not None:
        sink.append((tuple(buf[0:4]), tuple(buf[4:8])))


if __name__ == "__main__":
    main()
