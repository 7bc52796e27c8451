#!/bin/bash
# tools/sweep_duplex.sh [PCTS] [STEPS] -- tools/ab_duplex.py (sequential vs duplex, one
# process each) over the duplex decrypt's pool share (CYAES_DUPLEX_DYN_PCT) and range
# size (CYAES_DEC_RANGE_STEPS), configs B and C; output under gpurun_out/${OUT:-r05h}.
set -e
O=gpurun_out/${OUT:-r05h}; mkdir -p $O
for pct in ${1:-10 25 50}; do for rs in ${2:-2 4 8 16}; do
  timeout -k 10 120 python tools/ab_duplex.py --payloads 1048576 --payload-bytes 1472 --passes 32 --rounds 4 --lib cyclone_amd/libcyaes.so:CYAES_DUPLEX_DYN_PCT=$pct:CYAES_DEC_RANGE_STEPS=$rs > $O/B_p${pct}_r${rs}.txt 2>&1
  [ -n "$NOC" ] || timeout -k 10 120 python tools/ab_duplex.py --passes 6 --rounds 3 --lib cyclone_amd/libcyaes.so:CYAES_DUPLEX_DYN_PCT=$pct:CYAES_DEC_RANGE_STEPS=$rs > $O/C_p${pct}_r${rs}.txt 2>&1
done; done
