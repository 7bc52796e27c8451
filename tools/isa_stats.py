#!/usr/bin/env python3
"""tools/isa_stats.py -- per-kernel ISA statistics of the built kernel objects.

The device code of each build/cyaes_*kernels.o (its .hip_fatbin section,
unbundled for gfx950) disassembled with the ROCm LLVM tools; per kernel: the
instruction count, LDS reads (ds_read*: the AES table lookups), s_waitcnt,
scratch instructions (spills) and v_readlane / v_writelane (SGPR spills).
An LDS-bound step issues its 640 lookups in bursts; a schedule that lost them
shows as s_waitcnt per LDS read going from ~0.2 to ~0.4+ (r05: the strided
decrypt's lost schedule; r06: a runtime branch in the flat decrypt, DESIGN.md
§8), which tests/test_isa.py guards on CPU.

usage: python tools/isa_stats.py [--build build]
"""
import argparse
import collections
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
TUS = ("cyaes_kernels", "cyaes_enc_kernels", "cyaes_dec_kernels", "cyaes_duplex_kernels", "cyaes_ragged_kernels",
       "cyaes_batch_kernels")


def disassemble(obj, tmp):
    """gfx950 disassembly of a HIP object's device code."""
    fat, junk, dev = (os.path.join(tmp, n) for n in ("fat.bin", "junk.o", "dev.co"))
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, obj, junk], check=True,
                   capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + fat,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + dev], check=True, capture_output=True)
    return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", dev], check=True, capture_output=True,
                          text=True).stdout


def kernels(asm):
    """{mangled kernel name: Counter of mnemonics}."""
    out = {}
    heads = list(re.finditer(r"\n[0-9a-f]{16} <(_Z\S+)>:\n", asm))
    for i, m in enumerate(heads):
        body = asm[m.end():heads[i + 1].start() if i + 1 < len(heads) else len(asm)]
        ops = collections.Counter()
        for line in body.split("\n"):
            t = line.split("//")[0].strip()
            if t and not t.startswith("<") and not re.match(r"^[0-9a-f]+ <", t):
                ops[t.split()[0]] += 1
        out[m.group(1)] = ops
    return out


def stats(build=None):
    """{(tu, kernel): dict(insts, lds, waitcnt, scratch, lane_spill)} over the built objects
    (missing objects are skipped)."""
    build = build or os.path.join(ROOT, "build")
    res = {}
    with tempfile.TemporaryDirectory() as tmp:
        for tu in TUS:
            obj = os.path.join(build, tu + ".o")
            if not os.path.exists(obj):
                continue
            for name, ops in kernels(disassemble(obj, tmp)).items():
                res[(tu, name)] = {
                    "insts": sum(ops.values()),
                    "lds": sum(v for k, v in ops.items() if k.startswith("ds_read")),
                    "waitcnt": ops["s_waitcnt"],
                    "scratch": sum(v for k, v in ops.items() if k.startswith("scratch_")),
                    "lane_spill": ops["v_readlane_b32"] + ops["v_writelane_b32"],
                }
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", default=None)
    args = ap.parse_args()
    for (tu, name), s in sorted(stats(args.build).items()):
        print("%-22s %-70s insts %6d lds %5d waitcnt %4d (%.2f/lds) scratch %3d lane %4d" % (
            tu, name[:70], s["insts"], s["lds"], s["waitcnt"], s["waitcnt"] / max(1, s["lds"]), s["scratch"],
            s["lane_spill"]))


if __name__ == "__main__":
    main()
