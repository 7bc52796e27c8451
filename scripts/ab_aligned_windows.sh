#!/bin/bash
# A/B: ragged lane encrypt storing 16-B aligned windows (aw1) vs 4-B aligned
# blocks (base), then the GPU parity tests that check gaps/headers with aw1 as
# the library (box copy only).
set -u
O=gpurun_out/aw; mkdir -p $O
L="build/variants/base.so build/variants/aw1.so"
{
echo "== relay layouts, 1 M x 1472"; timeout -k 10 200 python tools/ab_relay_layout.py --lib $L --rounds 9 || exit 1
echo "== relay layouts, 65536 x 65280 (lane kernel forced)"; CYAES_QUAD_MAX_CHAINS=0 timeout -k 10 200 python tools/ab_relay_layout.py --lib $L --n 65536 --pb 65280 --rounds 5 --layouts contig_out,relay_out,relay_inplace || exit 1
echo "== relay layouts, 1 M x 1472 (reversed)"; timeout -k 10 200 python tools/ab_relay_layout.py --lib build/variants/aw1.so build/variants/base.so --rounds 9 --layouts relay_inplace,relay_out,contig_inplace || exit 1
} > $O/ab.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.txt | tail -40; [ $rc -ne 0 ] && exit $rc
cp build/variants/aw1.so cyclone_amd/libcyaes.so
CYAES_SWEEP_CASES=600 timeout -k 10 300 python -u -m pytest tests/test_gpu_sweep.py tests/test_batcher.py tests/test_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_aw1.txt 2>&1
rc=$?; tail -3 $O/pytest_aw1.txt; exit $rc
