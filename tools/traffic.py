"""Turns rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE csvs of `bench.py` (config C)
into profiles/traffic.json, the per-launch HBM traffic bench.py reports as
roofline.traffic.

Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): counters are in kB
(x1024); FETCH_SIZE on gfx950 counts half the bytes (x2).
usage: python tools/traffic.py FETCH_DIR WRITE_DIR [--out profiles/traffic.json]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ALGO = 2 * 262144 * 65536     # config C: read N + write N bytes per launch
NOTE = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bench.py config E with 2 passes (config "
        "C-sized encrypt, duplex and decrypt launches); "
        "FETCH_SIZE x2 per the gfx950 calibration, x1024 kB->B")


def per_launch_kb(d, counter):
    """Mean counter value (kB) per dispatch, for each AES kernel."""
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not path:
        raise SystemExit(f"no counter_collection.csv under {d}")
    sums = defaultdict(float)
    disp = defaultdict(set)
    with open(path[0]) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"]
            kind = ("encrypt" if "k_encrypt" in name else "decrypt" if "k_decrypt" in name else
                    "duplex" if "k_duplex" in name else None)
            if kind is None:
                continue
            sums[kind] += float(row["Counter_Value"])
            disp[kind].add(row["Dispatch_Id"])
    return {k: sums[k] / len(disp[k]) for k in sums}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--out", default="profiles/traffic.json")
    a = ap.parse_args()
    fetch = per_launch_kb(a.fetch_dir, "FETCH_SIZE")
    write = per_launch_kb(a.write_dir, "WRITE_SIZE")
    out = {"C": {}}
    for k in [k for k in ("encrypt", "decrypt", "duplex") if k in fetch and k in write]:
        fb = int(round(fetch[k] * 1024 * 2))
        wb = int(round(write[k] * 1024))
        out["C"][k] = {
            "bytes_per_launch": fb + wb, "fetch_bytes": fb, "write_bytes": wb,
            "algorithmic_bytes": ALGO * (2 if k == "duplex" else 1),
            "ratio": round((fb + wb) / (ALGO * (2 if k == "duplex" else 1)), 4),
            "raw": {"FETCH_SIZE_kB_per_launch": fetch[k], "WRITE_SIZE_kB_per_launch": write[k]},
            "note": NOTE,
        }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v["ratio"] for k, v in out["C"].items()}))


if __name__ == "__main__":
    main()
