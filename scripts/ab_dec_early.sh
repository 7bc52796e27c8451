#!/bin/bash
# A/B: flat decrypt with the next step's loads before this step's stores and the
# progress atomic's answer used after the rounds (el1; atomic optimizer off so the
# atomic is not broadcast at once), the atomic optimizer off alone (ao0), the
# current build (base).  Plus ragged-encrypt store offsets (base vs onepf).
set -u
O=gpurun_out/dec_early; mkdir -p $O
{
echo "== config C"; timeout -k 10 200 python tools/ab.py build/variants/base.so build/variants/el1.so build/variants/ao0.so --rounds 8 || exit 1
echo "== config B"; timeout -k 10 200 python tools/ab.py build/variants/base.so build/variants/el1.so build/variants/ao0.so --rounds 10 --payloads 1048576 --payload-bytes 1472 || exit 1
echo "== config C (reversed)"; timeout -k 10 200 python tools/ab.py build/variants/ao0.so build/variants/el1.so build/variants/base.so --rounds 8 || exit 1
echo "== relay encrypt, lane kernel: store offsets (base) vs onepf"; timeout -k 10 200 python tools/ab_relay_layout.py --lib build/variants/base.so build/variants/onepf.so --layouts relay_inplace,relay_out,contig_out || exit 1
} > $O/ab.txt 2>&1
rc=$?; grep -v "amdgpu.ids" $O/ab.txt | tail -30; exit $rc
