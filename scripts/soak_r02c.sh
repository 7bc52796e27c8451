#!/bin/bash
# 2000-case randomized parity soak of the current build, then the GPU suite again.
set -u
O=gpurun_out/soak_c; mkdir -p $O
CYAES_SWEEP_CASES=2000 timeout -k 10 300 python -u -m pytest tests/test_gpu_sweep.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/sweep_2000.txt 2>&1
rc=$?; tail -2 $O/sweep_2000.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -2 $O/pytest_gpu.txt; exit $rc
