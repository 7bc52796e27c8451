#!/bin/bash
# A/B: encrypt next-chunk prefetch as one load path (onepf, no wait on the
# previous chunk's stores) vs the r02 two-path tail prefetch (twopf).
set -u
O=gpurun_out/onepf; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -2 $O/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
L="build/variants/onepf.so build/variants/twopf.so"
R="build/variants/twopf.so build/variants/onepf.so"
{
echo "== config C"; timeout -k 10 200 python tools/ab.py $L --rounds 8 || exit 1
echo "== config B"; timeout -k 10 200 python tools/ab.py $L --rounds 10 --payloads 1048576 --payload-bytes 1472 || exit 1
echo "== relay streams, lane kernel forced"; CYAES_QUAD_MAX_CHAINS=0 timeout -k 10 200 python tools/ab_relay_layout.py --lib $L --layouts contig_out,relay_out,relay_inplace || exit 1
echo "== config C (reversed order)"; timeout -k 10 200 python tools/ab.py $R --rounds 8 || exit 1
echo "== config B (reversed order)"; timeout -k 10 200 python tools/ab.py $R --rounds 10 --payloads 1048576 --payload-bytes 1472 || exit 1
} > $O/ab.txt 2>&1
rc=$?; cat $O/ab.txt | grep -v "^\s*$" | tail -40; exit $rc
