#!/usr/bin/env python3
"""tools/pmc_kernels.py -- mean counter value per kernel launch from rocprofv3
--pmc output directories (run_counter_collection.csv), for the AES kernels.

usage: python tools/pmc_kernels.py DIR [DIR ...] [--match k_decrypt_flat]
Prints, per directory, kernel (name shortened), launches, counter and mean value
per launch (FETCH_SIZE / WRITE_SIZE in kB as rocprofv3 reports them; FETCH_SIZE
x2 and kB x1024 give bytes on gfx950, tools/traffic.py)."""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="k_")
    args = ap.parse_args()
    for d in args.dirs:
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        acc = collections.defaultdict(list)
        for f in files:
            for row in csv.DictReader(open(f)):
                name = row["Kernel_Name"]
                if args.match not in name:
                    continue
                short = name.replace("void ", "").replace("cyaes::(anonymous namespace)::", "").split("(")[0]
                acc[(short, row["Counter_Name"])].append(float(row["Counter_Value"]))
        for (k, c), v in sorted(acc.items()):
            print("%-40s %-60s %4d launches  %-11s mean %.1f" % (os.path.basename(d.rstrip("/")), k, len(v), c,
                                                                  sum(v) / len(v)))


if __name__ == "__main__":
    main()
