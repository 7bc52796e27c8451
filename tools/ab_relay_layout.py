#!/usr/bin/env python3
"""tools/ab_relay_layout.py -- where ragged / strided encrypt and decrypt lose time on relay streams.

Times cyaes_gpu_encrypt_ragged, then cyaes_gpu_decrypt_ragged of its output (--api strided:
cyaes_gpu_{en,de}crypt_strided)
(in place, or back into the source stream), on N equal payloads under layouts that differ in
one property at a time: packet stride (payload + header bytes), payload offset
inside the packet (12 = relay, 16 = 16-B aligned) and in place vs a separate
output stream.  usage: python tools/ab_relay_layout.py [--n 1048576] [--pb 1472]
[--lib a.so[:ENV=V] [b.so ...]] [--layouts relay_inplace,...]  (several libs: interleaved per round, one process)"""
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
    ap.add_argument("--lib", nargs="*", default=None)
    ap.add_argument("--layouts", default=None, help="comma-separated subset of the layout labels")
    ap.add_argument("--api", choices=["ragged", "strided"], default="ragged",
                    help="ragged entry points (device offset / size lists) or the strided ones")
    args = ap.parse_args()
    import numpy as np
    import torch
    import cyclone_amd as ca
    libs = args.lib or [None]
    ctxs = []
    for spec in libs:  # path[:ENV=V...]: the environment the context is created under (CYAES_* switches)
        path, *envs = (spec or "").split(":")
        saved = {}
        for kv in envs:
            k, v = kv.split("=", 1)
            saved[k] = os.environ.get(k)
            os.environ[k] = v
        ctxs.append(ca.GpuContext(0, lib=ca.load_library(os.path.abspath(path)) if path else None))
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    for c in ctxs:
        c.set_keys(bytes(range(16)))
    c = ctxs[0]
    s = torch.cuda.current_stream()
    n, pb = args.n, args.pb
    pt = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
    c.fill_synthetic(pt, 0, n, pb, 0x5EEDC1C1)
    ref = torch.empty_like(pt)
    c.encrypt_uniform(pt, ref, n, pb, stream=s.cuda_stream)
    nb = torch.full((n,), pb, dtype=torch.int32, device="cuda")
    # (label, header bytes before the payload, packet stride, in place)
    layouts = [("contig_out", 0, pb, False), ("contig_inplace", 0, pb, True),
               ("hdr16_out", 16, pb + 16, False), ("hdr16_inplace", 16, pb + 16, True),
               ("hdr12_s1488_out", 12, pb + 16, False), ("hdr12_s1488_inplace", 12, pb + 16, True),
               ("relay_out", 12, pb + 12, False), ("relay_inplace", 12, pb + 12, True),
               # r03: alignment alone (contiguous payloads shifted off 16/32 B) vs stride alone
               ("contig_off4_inplace", 4, pb, True), ("contig_off16_inplace", 16, pb, True),
               ("contig_off32_inplace", 32, pb, True), ("s1536_off0_inplace", 0, 1536, True),
               ("s1536_off12_inplace", 12, 1536, True), ("s1536_off16_inplace", 16, 1536, True)]
    if args.layouts:
        keep = args.layouts.split(",")
        layouts = [ly for ly in layouts if ly[0] in keep]
    for label, hdr, stride, inplace in layouts:
        src = torch.zeros(n * stride + 64, dtype=torch.uint8, device="cuda")
        fill = lambda: src[hdr: hdr + n * stride].view(n, stride)[:, :pb].copy_(pt.view(n, pb))
        fill()
        dst = src if inplace else torch.zeros_like(src)
        off = torch.from_numpy(np.arange(n, dtype=np.uint64) * stride + hdr).to("cuda")
        ts = [[] for _ in ctxs]
        td = [[] for _ in ctxs]
        ok = [True for _ in ctxs]
        for r in range(args.rounds + 1):
            for k, ck in enumerate(ctxs):
                if inplace:
                    fill()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                if args.api == "strided":
                    ck.encrypt_strided(src, dst, hdr, stride, n, pb, stream=s.cuda_stream)
                else:
                    ck.encrypt_ragged(src, dst, off, nb, n, stream=s.cuda_stream)
                e1.record(s)
                torch.cuda.synchronize()
                if r:
                    ts[k].append(e0.elapsed_time(e1))
                ok[k] = ok[k] and torch.equal(dst[hdr: hdr + n * stride].view(n, stride)[:, :pb].reshape(-1), ref)
                # decrypt the stream just encrypted: in place, or into the (plaintext) source stream
                back = dst if inplace else src
                e0.record(s)
                if args.api == "strided":
                    ck.decrypt_strided(dst, back, hdr, stride, n, pb, stream=s.cuda_stream)
                else:
                    ck.decrypt_ragged(dst, back, off, nb, n, stream=s.cuda_stream)
                e1.record(s)
                torch.cuda.synchronize()
                if r:
                    td[k].append(e0.elapsed_time(e1))
                ok[k] = ok[k] and torch.equal(back[hdr: hdr + n * stride].view(n, stride)[:, :pb].reshape(-1), pt)
        for k, p in enumerate(libs):
            print("%-22s %8d x %5d B stride %5d: enc %.4f ms (min %.4f) dec %.4f ms (min %.4f)  %s  %s" %
                  (label, n, pb, stride, statistics.median(ts[k]), min(ts[k]), statistics.median(td[k]), min(td[k]),
                   "ok" if ok[k] else "MISMATCH", p or ""), flush=True)
        del src, dst
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
