#!/usr/bin/env python3
"""tools/isa_mix.py -- instruction mix of one kernel in a hipcc -S listing.

usage: python tools/isa_mix.py listing.s SUBSTRING [top]
       python tools/isa_mix.py listing.s SUBSTRING --blocks   (per basic block with LDS reads:
       instructions, ds_read, s_waitcnt, SGPR-spill lane moves, global loads / stores)
(listing: hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S ...)"""
import collections
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3] != "--blocks" else 16
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(key), l))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    if len(sys.argv) > 3 and sys.argv[3] == "--blocks":
        blocks, cur = [], None
        for l in lines[start:end + 1]:
            if re.match(r"^\.LBB\S*:", l) or cur is None:
                cur = {"label": l.split(":")[0] if l.startswith(".LBB") else "entry", "n": collections.Counter()}
                blocks.append(cur)
            m = re.match(r"^\s+([sv]_\w+|ds_\w+|global_\w+|buffer_\w+|scratch_\w+)", l)
            if m:
                op = m.group(1)
                cur["n"]["insts"] += 1
                for k in ("ds_read", "s_waitcnt", "v_writelane", "v_readlane", "global_load", "global_store",
                          "global_atomic", "scratch_", "s_setprio"):
                    if op.startswith(k):
                        cur["n"][k] += 1
        for b in blocks:
            n = b["n"]
            if n["ds_read"] or n["v_writelane"] or n["scratch_"]:
                print("%-14s insts %5d ds_read %4d waitcnt %4d writelane %3d readlane %3d gload %3d gstore %3d "
                      "atomic %d scratch %d" % (b["label"], n["insts"], n["ds_read"], n["s_waitcnt"], n["v_writelane"],
                                                n["v_readlane"], n["global_load"], n["global_store"],
                                                n["global_atomic"], n["scratch_"]))
        return
    c = collections.Counter()
    for l in lines[start:end + 1]:
        m = re.match(r"^\s+([sv]_\w+|ds_\w+|global_\w+|buffer_\w+)", l)
        if m:
            c[m.group(1)] += 1
    for k, v in c.most_common(top):
        print("%6d %s" % (v, k))


if __name__ == "__main__":
    main()
