#!/bin/bash
# r02 profiling session (GPU box): rocprofv3 kernel-trace stats of the headline
# bench (config E), PMC traffic passes (config C = one E pass), counter list.
# Output: gpurun_out/$TAG/.  usage: scripts/gpu_profile_r02.sh TAG
set -u
TAG=${1:-r02}
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
cd /tmp
step counters 60 rocprofv3 -L
step rocprof_stats 300 rocprofv3 --kernel-trace --stats -d "$O/rocprof" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --packet-configs none --relay-stream 0
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" --config C --steps 2 --warmup 0 --no-cpu --no-verify --no-clock --packet-configs none --relay-stream 0
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" --config C --steps 2 --warmup 0 --no-cpu --no-verify --no-clock --packet-configs none --relay-stream 0
echo "[gpu] done"
