#!/bin/bash
# A/B: quad encrypt with the single prefetch path (q1) vs the r02 loop (q0),
# on the latency-bound batch sizes the quad kernel serves.
set -u
O=gpurun_out/quad_onepf; mkdir -p $O
L="build/variants/q1.so build/variants/q0.so"
{
for sz in "1 1472" "64 1472" "4096 1024" "16384 1472" "65535 1472" "16384 65536" "65535 65536"; do
  set -- $sz
  echo "== $1 x $2"; timeout -k 10 200 python tools/ab.py $L --rounds 12 --payloads $1 --payload-bytes $2 || exit 1
done
echo "== relay stream 65536 packets"; timeout -k 10 200 python tools/ab_relay_layout.py --lib $L --n 65536 --layouts relay_inplace,relay_out || exit 1
echo "== 16384 x 1472 (reversed)"; timeout -k 10 200 python tools/ab.py build/variants/q0.so build/variants/q1.so --rounds 12 --payloads 16384 --payload-bytes 1472 || exit 1
} > $O/ab.txt 2>&1
rc=$?; grep -v "amdgpu.ids" $O/ab.txt | tail -40; exit $rc
