#!/usr/bin/env python3
"""tools/isa_mix.py -- instruction mix of one kernel in a hipcc -S listing.

usage: python tools/isa_mix.py listing.s SUBSTRING [top]
(listing: hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S ...)"""
import collections
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(key), l))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    c = collections.Counter()
    for l in lines[start:end + 1]:
        m = re.match(r"^\s+([sv]_\w+|ds_\w+|global_\w+|buffer_\w+)", l)
        if m:
            c[m.group(1)] += 1
    for k, v in c.most_common(top):
        print("%6d %s" % (v, k))


if __name__ == "__main__":
    main()
