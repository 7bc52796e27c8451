#!/bin/bash
# r02 end-of-round check on the GPU box: full GPU suite, smoke(), the default
# bench line (config E + packet configs B/D + CPU baseline), then the profiling
# session (rocprof kernel stats of the bench, PMC traffic passes).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/final2
mkdir -p "$O"
cd "$R"
timeout -k 10 420 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > "$O/pytest_gpu.txt" 2>&1
rc=$?; tail -2 "$O/pytest_gpu.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.txt" 2>&1
rc=$?; tail -1 "$O/smoke.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; cut -c1-300 "$O/bench.json"; [ $rc -ne 0 ] && { tail -5 "$O/bench.err"; exit $rc; }
bash scripts/gpu_profile_r02.sh final2_prof
