#!/bin/bash
# PMC FETCH_SIZE / WRITE_SIZE per relay-layout decrypt (one rocprofv3 pass per counter and layout)
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05z; mkdir -p $O
cd /tmp; export TMPDIR=/tmp
for ly in relay_inplace contig_inplace relay_out contig_out; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d $O/${ly}_$c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ab_relay_layout.py --api strided --rounds 3 --layouts $ly > $O/${ly}_$c.log 2>&1
  done
done
