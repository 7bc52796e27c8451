#!/bin/bash
# One GPU-box session: parity tests, bench (+cpu baseline), the other configs,
# end-to-end (host memory) bench and link probe, rocprofv3 kernel-trace stats,
# PMC traffic passes.  Output: gpurun_out/$TAG/
# usage: scripts/gpu_profile.sh TAG
set -u
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[gpu] $name"
  timeout -k 10 "$secs" "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "[gpu] $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$O/$name.err"; exit $rc; fi
}
cd "$R"
step pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
step bench 400 python bench.py --steps 10 --warmup 2
step bench_B 200 python bench.py --config B --steps 20 --warmup 2 --no-cpu --packet-configs none
step bench_D 200 python bench.py --config D --steps 20 --warmup 2 --no-cpu --packet-configs none
step bench_A 200 python bench.py --config A --steps 20 --warmup 2 --no-cpu --packet-configs none
step linkprobe 200 python tools/linkprobe.py
step bench_e2e_pinned 300 python bench_e2e.py --host pinned
step bench_e2e_pageable 300 python bench_e2e.py --host pageable
cd /tmp
step rocprof_stats 400 rocprofv3 --kernel-trace --stats -d "$O/rocprof" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu --packet-configs none
step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu --no-verify --packet-configs none
step pmc_write 400 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu --no-verify --packet-configs none
echo "[gpu] done"
