#!/usr/bin/env python3
"""tools/pmc_summary.py -- per-kernel averages of rocprofv3 --pmc counter csvs,
with the derived VALU / LDS utilisation figures.

usage: python tools/pmc_summary.py DIR [DIR...] [--match k_encrypt,k_decrypt,k_bs]"""
import argparse
import csv
import re
import glob
import os
from collections import defaultdict

NUM_CUS = 256


def load(d):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    sums = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for p in path:
        with open(p) as f:
            for row in csv.DictReader(f):
                k = row["Kernel_Name"]
                sums[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add(row["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in cs.items()} for k, cs in sums.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="k_encrypt,k_decrypt,k_bs")
    a = ap.parse_args()
    keys = a.match.split(",")
    merged = defaultdict(dict)
    for d in a.dirs:
        for k, cs in load(d).items():
            merged[k].update(cs)
    for k, c in merged.items():
        if not any(m in k for m in keys):
            continue
        m = re.search(r"(k_\w+(<[^>]*>)?)", k)
        short = m.group(1) if m else k[:60]
        print("== %s" % short)
        for n in sorted(c):
            print("   %-24s %.6g" % (n, c[n]))
        g = c.get("GRBM_GUI_ACTIVE")
        if g:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs: kernel cycles = g / 8
            cyc = g / 8
            if "SQ_ACTIVE_INST_VALU" in c:
                # quad-cycles of VALU issue over the 4 SIMDs of every CU
                print("   VALU busy (quad-cycles x4 / SIMD cycles)  %.3f" % (4 * c["SQ_ACTIVE_INST_VALU"] / (4 * NUM_CUS * cyc)))
            if "SQ_LDS_IDX_ACTIVE" in c:
                print("   LDS index active / CU cycles              %.3f" % (c["SQ_LDS_IDX_ACTIVE"] / (NUM_CUS * cyc)))
        if c.get("SQ_INSTS_LDS"):
            print("   VALU insts per LDS inst        %.3f" % (c["SQ_INSTS_VALU"] / c["SQ_INSTS_LDS"]))
        if "SQ_ACTIVE_INST_VALU2" in c and "SQ_ACTIVE_INST_VALU" in c:
            print("   VALU2 / VALU quad-cycles       %.3f" % (c["SQ_ACTIVE_INST_VALU2"] / c["SQ_ACTIVE_INST_VALU"]))


if __name__ == "__main__":
    main()
