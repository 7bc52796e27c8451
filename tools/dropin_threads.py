#!/usr/bin/env python3
"""tools/dropin_threads.py -- synchronous drop-in (cyclone::Rijndael-shaped
calls, iv = nullptr as the relay passes) from T threads at once, as the
relay's per-core looper threads call it (relay_local.cpp:475): total calls/s
and GiB/s per thread count.  ctypes releases the GIL around each call.
usage: python tools/dropin_threads.py [--size 1472] [--seconds 2] [--threads 1,2,4,8,16,32]"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1472)
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--threads", default="1,2,4,8,16,32")
    ap.add_argument("--op", default="encrypt", choices=["encrypt", "decrypt"])
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's, see cyclone_amd)
    import cyclone_amd as ca
    for T in [int(x) for x in args.threads.split(",")]:
        objs = [ca.Rijndael(bytes((t * 16 + i) & 255 for i in range(16))) for t in range(T)]
        buf = bytes(range(256)) * (args.size // 256 + 1)
        buf = buf[:args.size]
        for o in objs:
            getattr(o, args.op)(buf)  # warm-up
        counts = [0] * T
        stop = threading.Event()

        def work(t):
            f = getattr(objs[t], args.op)
            n = 0
            while not stop.is_set():
                f(buf)
                n += 1
            counts[t] = n

        th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        time.sleep(args.seconds)
        stop.set()
        for x in th:
            x.join()
        el = time.perf_counter() - t0
        calls = sum(counts)
        print(json.dumps({"metric": "drop-in %s calls/s" % args.op, "size": args.size, "threads": T,
                          "calls_per_s": round(calls / el), "gibs": round(calls * args.size / el / 2**30, 4),
                          "us_per_call_per_thread": round(el * 1e6 * T / max(1, calls), 1)}), flush=True)


if __name__ == "__main__":
    main()
