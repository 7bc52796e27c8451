#!/bin/bash
# Ragged encrypt: lane kernel (one lane per chain) vs quad kernel on relay
# streams of n packets, after the single-path prefetch (scripts/ab_onepf.sh).
# The kernel choice is per process (CYAES_QUAD_MAX_CHAINS), so processes alternate.
set -u
O=gpurun_out/ragged_switch; mkdir -p $O
{
for n in 16384 65536 131072 262144 524288 1048576 2097152; do
  for rep in 1 2; do
    for k in lane quad; do
      if [ $k = lane ]; then q=0; else q=1000000000000; fi
      echo "-- n=$n $k rep $rep"
      CYAES_QUAD_MAX_CHAINS=$q timeout -k 10 120 python tools/ab_relay_layout.py --n $n --rounds 7 --layouts relay_inplace,relay_out || exit 1
    done
  done
done
} > $O/switch.txt 2>&1
rc=$?; grep -v "amdgpu.ids" $O/switch.txt | tail -70; exit $rc
