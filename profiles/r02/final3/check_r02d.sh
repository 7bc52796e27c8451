#!/bin/bash
# Re-check after an illegal-address report at sweep case 69 (previous call): the
# sweep alone with kernels serialized (a fault then names its launch), then the
# rest of the GPU suite, smoke and bench.  Stops at the first failure.
set -u
O=gpurun_out/check_d; mkdir -p $O
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_sweep.py -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest_sweep.txt 2>&1
rc=$?; tail -3 $O/pytest_sweep.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -2 $O/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
rc=$?; tail -1 $O/smoke.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; cut -c1-300 $O/bench.json; exit $rc
