#!/bin/bash
# A/B: uniform lane encrypt prefetching the lane's next payload (nx1) vs base.
set -u
O=gpurun_out/nx; mkdir -p $O
L="build/variants/base.so build/variants/nx1.so"
R="build/variants/nx1.so build/variants/base.so"
{
echo "== config B"; timeout -k 10 200 python tools/ab.py $L --rounds 12 --payloads 1048576 --payload-bytes 1472 || exit 1
echo "== config D"; timeout -k 10 200 python tools/ab.py $L --rounds 12 --payloads 1048576 --payload-bytes 1472 --ppk 256 || exit 1
echo "== 1 M x 1024"; timeout -k 10 200 python tools/ab.py $L --rounds 12 --payloads 1048576 --payload-bytes 1024 || exit 1
echo "== config C"; timeout -k 10 200 python tools/ab.py $L --rounds 6 || exit 1
echo "== config B (reversed)"; timeout -k 10 200 python tools/ab.py $R --rounds 12 --payloads 1048576 --payload-bytes 1472 || exit 1
} > $O/ab.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.txt | tail -20; exit $rc
