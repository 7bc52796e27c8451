#!/bin/bash
# Round-end shape check (as the driver runs it): the GPU suite, smoke(), the default bench line.
set -u
O=gpurun_out/${1:-check_e}; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -2 $O/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
rc=$?; tail -1 $O/smoke.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; cut -c1-300 $O/bench.json; exit $rc
