#!/usr/bin/env python3
"""tools/resusage.py -- per-kernel register use of one kernel translation unit.

Compiles FILE for gfx950 with -Rpass-analysis=kernel-resource-usage (extra
hipcc flags after the file) and prints one line per kernel: VGPRs, AGPRs,
SGPRs, spills, LDS, occupancy.  usage: python tools/resusage.py FILE [FLAGS...]"""
import re
import subprocess
import sys
import tempfile

ROOT = __file__.rsplit("/tools/", 1)[0]


def main():
    src, flags = sys.argv[1], sys.argv[2:]
    with tempfile.TemporaryDirectory() as d:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I" + ROOT + "/include",
               "-I" + ROOT + "/cyclone_amd/csrc", "-Rpass-analysis=kernel-resource-usage", "-c", src,
               "-o", d + "/x.o"] + flags
        err = subprocess.run(cmd, capture_output=True, text=True).stderr
    cur, rows = None, []
    for ln in err.splitlines():
        m = re.search(r"remark: (?:\s*)(Function Name|VGPRs|AGPRs|TotalSGPRs|SGPRs Spill|VGPRs Spill|"
                      r"LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+)", ln)
        if not m:
            continue
        k, v = m.groups()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for r in rows:
        name = r["name"]
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        name = name.replace("cyaes::(anonymous namespace)::", "").replace("HIP_vector_type<unsigned int, 4u>", "uint4")
        print("%-60s vgpr %4s agpr %3s sgpr %4s spill s/v %3s/%-3s lds %6s occ %s" % (
            name[:60], r.get("VGPRs"), r.get("AGPRs"), r.get("TotalSGPRs"), r.get("SGPRs Spill"),
            r.get("VGPRs Spill"), r.get("LDS Size [bytes/block]"), r.get("Occupancy [waves/SIMD]")))


if __name__ == "__main__":
    main()
