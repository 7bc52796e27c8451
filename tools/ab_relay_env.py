#!/usr/bin/env python3
"""tools/ab_relay_env.py -- interleaved A/B of context settings (environment
variables read at context creation) on relay streams, in ONE process.

usage: python tools/ab_relay_env.py [--rounds 8] [--what duplex,mixed,ragged] SPEC [SPEC ...]
  SPEC: NAME=VALUE[:NAME=VALUE...] or "base" (no settings).
  duplex: config B's payloads as two relay streams (offset 12, stride 1,484);
          per variant the two strided calls and one cyaes_gpu_duplex_strided.
  mixed:  bench.py's mixed-size relay stream (mixed_stream_layout) through the
          ragged entry points, encrypt and decrypt in place.
  ragged: config B's relay stream through the ragged entry points.
  mixdup: the mixed stream encrypted while a second copy is decrypted:
          the two ragged calls, cyaes_gpu_duplex_ragged, and the duplex with a
          one-packet decrypt (the packed encrypt alone).
Prints per variant the median / min ms of each timed call and checks every
variant's output against the first one's.
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("specs", nargs="+")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--what", default="duplex,mixed")
    ap.add_argument("--ragged-n", type=int, default=0, help="ragged: packets (0 = config B's 1 M)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import cyclone_amd as ca

    ctxs = []
    for spec in args.specs:
        env = {} if spec == "base" else dict(kv.split("=", 1) for kv in spec.split(":"))
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        c = ca.GpuContext(0)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        c.set_keys(bytes(range(16)))
        ctxs.append((spec, c))
    s = torch.cuda.current_stream()
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

    def timed(fn):
        a, b = ev(), ev()
        a.record(s)
        fn()
        b.record(s)
        return a, b

    what = args.what.split(",")
    n, pb = bench.CONFIGS["B"][0], bench.CONFIGS["B"][1]
    hdr, stride = 12, pb + 12
    if "duplex" in what or "ragged" in what:
        pt = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
        ctxs[0][1].fill_synthetic(pt, 0, n, pb, bench.PLAINTEXT_SEED)
        b1 = torch.full((n * stride + 16,), 0xA5, dtype=torch.uint8, device="cuda")
        b2 = torch.full_like(b1, 0xA5)
        v1, v2 = b1[: n * stride].view(n, stride), b2[: n * stride].view(n, stride)
        d_off = torch.arange(n, dtype=torch.int64, device="cuda") * stride + hdr
        d_nb = torch.full((n,), pb, dtype=torch.int32, device="cuda")
    if "mixed" in what or "mixdup" in what:
        offs, nbs, alloc = bench.mixed_stream_layout(n * pb)
        mn = int(offs.size)
        mbuf = torch.empty(alloc, dtype=torch.uint8, device="cuda")
        m_off = torch.from_numpy(offs.astype(np.int64)).to("cuda")
        m_nb = torch.from_numpy(nbs.astype(np.int32)).to("cuda")
        if "mixdup" in what:
            mbuf2 = torch.empty_like(mbuf)
    res = {spec: {} for spec, _ in ctxs}
    ref_out = {}
    for r in range(args.rounds + 1):
        for spec, c in ctxs:
            evs = {}
            if "duplex" in what:
                if r == 0:  # parity once: the duplex equals the two calls
                    v1[:, hdr:hdr + pb] = pt.view(n, pb)
                    v2[:, hdr:hdr + pb] = pt.view(n, pb)
                    c.encrypt_strided(b2, b2, hdr, stride, n, pb)
                    c.encrypt_strided(b1, b1, hdr, stride, n, pb)
                    c.decrypt_strided(b2, b2, hdr, stride, n, pb)
                    out_two = (b1.clone(), b2.clone())
                    v1[:, hdr:hdr + pb] = pt.view(n, pb)
                    c.encrypt_strided(b2, b2, hdr, stride, n, pb)
                    c.duplex_strided(b1, b1, hdr, stride, n, pb, b2, b2, hdr, stride, n, pb)
                    torch.cuda.synchronize()
                    assert torch.equal(b1, out_two[0]) and torch.equal(b2, out_two[1]), spec
                    del out_two
                # Steady state, as bench.py times it: 6 back-to-back steps of each
                # form, the last 3 timed; the order of the two forms alternates per round.
                forms = [("two_calls", lambda: (c.encrypt_strided(b1, b1, hdr, stride, n, pb),
                                                c.decrypt_strided(b2, b2, hdr, stride, n, pb))),
                         ("duplex", lambda: c.duplex_strided(b1, b1, hdr, stride, n, pb, b2, b2, hdr, stride, n, pb))]
                if r % 2:
                    forms.reverse()
                for name, fn in forms:
                    for k in range(6):
                        e = timed(fn)
                        if k >= 3:
                            evs.setdefault(name, []).append(e)
            if "ragged" in what:  # the first args.ragged_n packets of the stream, equal sizes
                rn = args.ragged_n or n
                v1[:, hdr:hdr + pb] = pt.view(n, pb)
                for k in range(4):
                    ea = timed(lambda: c.encrypt_ragged(b1, b1, d_off, d_nb, rn))
                    da = timed(lambda: c.decrypt_ragged(b1, b1, d_off, d_nb, rn))
                    if k >= 2:
                        evs.setdefault("rag_enc", []).append(ea)
                        evs.setdefault("rag_dec", []).append(da)
            if "mixed" in what:
                c.fill_synthetic(mbuf, 0, alloc // 16, 16, bench.PLAINTEXT_SEED)
                if r == 0:  # parity once: every variant's ciphertext is the first one's
                    c.encrypt_ragged(mbuf, mbuf, m_off, m_nb, mn)
                    d = c.digest(mbuf, alloc)
                    ref_out.setdefault("mix", d)
                    assert d == ref_out["mix"], spec
                    c.decrypt_ragged(mbuf, mbuf, m_off, m_nb, mn)
                for k in range(4):
                    ea = timed(lambda: c.encrypt_ragged(mbuf, mbuf, m_off, m_nb, mn))
                    da = timed(lambda: c.decrypt_ragged(mbuf, mbuf, m_off, m_nb, mn))
                    if k >= 2:
                        evs.setdefault("mix_enc", []).append(ea)
                        evs.setdefault("mix_dec", []).append(da)
            if "mixdup" in what:
                c.fill_synthetic(mbuf, 0, alloc // 16, 16, bench.PLAINTEXT_SEED)
                c.fill_synthetic(mbuf2, 0, alloc // 16, 16, bench.PLAINTEXT_SEED)
                c.encrypt_ragged(mbuf2, mbuf2, m_off, m_nb, mn)
                if r == 0:  # parity once: the duplex gives the two calls' bytes
                    c.duplex_ragged(mbuf, mbuf, m_off, m_nb, mn, mbuf2, mbuf2, m_off, m_nb, mn)
                    d = (c.digest(mbuf, alloc), c.digest(mbuf2, alloc))
                    c.decrypt_ragged(mbuf, mbuf, m_off, m_nb, mn)
                    c.encrypt_ragged(mbuf2, mbuf2, m_off, m_nb, mn)
                    ref_out.setdefault("mixdup", d)
                    assert d == ref_out["mixdup"], spec
                forms = [("two_calls", lambda: (c.encrypt_ragged(mbuf, mbuf, m_off, m_nb, mn),
                                                c.decrypt_ragged(mbuf2, mbuf2, m_off, m_nb, mn))),
                         ("duplex", lambda: c.duplex_ragged(mbuf, mbuf, m_off, m_nb, mn, mbuf2, mbuf2, m_off, m_nb,
                                                            mn)),
                         ("packed_enc", lambda: c.duplex_ragged(mbuf, mbuf, m_off, m_nb, mn, mbuf2, mbuf2, m_off,
                                                                m_nb, 1))]
                if r % 2:
                    forms.reverse()
                for name, fn in forms:
                    for k in range(6):
                        e = timed(fn)
                        if k >= 3:
                            evs.setdefault(name, []).append(e)
            torch.cuda.synchronize()
            if r == 0:
                continue  # warm-up round
            for k, v in evs.items():
                for a, b in (v if isinstance(v, list) else [v]):
                    res[spec].setdefault(k, []).append(a.elapsed_time(b))
    for spec, d in res.items():
        print("%-48s %s" % (spec, " | ".join("%s med %.4f min %.4f" % (k, statistics.median(v), min(v))
                                              for k, v in d.items())))


if __name__ == "__main__":
    main()
