#!/bin/bash
# r02 (session 6) check on the GPU box: the new RCCL world-1 test first, then the
# full GPU suite, smoke() and the default bench line.  Optional arg: output subdir.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-check_c}
mkdir -p "$O"
cd "$R"
CYAES_TEST_RCCL=1 timeout -k 10 200 python -u -m pytest tests/test_config_e.py -m gpu -v --timeout 150 --timeout-method thread -k rccl > "$O/pytest_rccl.txt" 2>&1
rc=$?; tail -2 "$O/pytest_rccl.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > "$O/pytest_gpu.txt" 2>&1
rc=$?; tail -2 "$O/pytest_gpu.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.txt" 2>&1
rc=$?; tail -1 "$O/smoke.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; cut -c1-400 "$O/bench.json"; [ $rc -ne 0 ] && { tail -5 "$O/bench.err"; exit $rc; }
exit 0
