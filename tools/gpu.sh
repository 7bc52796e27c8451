#!/bin/bash
# tools/gpu.sh -- the one GPU-box runner (replaces round 2's per-experiment
# scripts/).  Runs the named steps in order under their own time limits and
# stops at the first failure; every step's output goes to gpurun_out/$OUT/.
#
# usage: tools/gpu.sh OUT STEP [STEP ...]
#   test       python -m pytest tests -m gpu (product build)
#   bounds     the same suite on the bounds-checked build (CYAES_LIBRARY=build/variants/bounds.so)
#   smoke      __graft_entry__.smoke()
#   soak       tests/test_gpu_sweep.py with CYAES_SWEEP_CASES=${SOAK:-2000}
#   bench      python bench.py (default: config E headline + packet configs + relay stream)
#   quickbench bench.py --steps 3 --warmup 1 (no CPU baseline)
#   profile    rocprofv3 --kernel-trace --stats of a short bench, then FETCH_SIZE / WRITE_SIZE PMC passes
#              (config E, 2 passes: an encrypt, a duplex and a decrypt launch of config C's size)
#   cfgtest    tests/test_config_e.py only (bench.py's own contract and multi-rank runs)
#   pytest:F   tests/F (a file or file::test), -m gpu
#   batchertest  tests/test_batcher.py only
#   batcher    build/bench_batcher SEAL / OPEN loads (host to host), zero-copy and bounce ($BB_ARGS appended)
#   hostlink   build/hostlink: kernel-driven packet gather/scatter over PCIe vs DMA
#   bb:ARGS    one build/bench_batcher run (ARGS comma-separated) with CYAES_BATCHER_PROFILE phases, to bb.txt
#   ab:A:B[:ARGS]  tools/ab.py on variant libraries build/variants/{A,B}.so, both orders
#                  (ARGS: extra ab.py arguments, commas for spaces)
#   abrelay:A:B    tools/ab_relay_layout.py on the two variants (relay stream layouts)
#   abenv:NAME=V[+NAME=V]:ARGS  tools/ab.py: the product library vs itself with those context env settings
set -u
OUT=${1:?usage: tools/gpu.sh OUT STEP...}
shift
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$OUT
mkdir -p "$O"
export TMPDIR=/tmp
PYT="python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread"

run() {  # run NAME SECONDS CMD...: output to $O/NAME.txt, stop the script on failure
  local name=$1 secs=$2
  shift 2
  echo "[gpu] $name: $*"
  timeout -k 10 "$secs" "$@" > "$O/$name.txt" 2>&1
  local rc=$?
  echo "[gpu] $name rc=$rc"
  tail -3 "$O/$name.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
}

for step in "$@"; do
  case $step in
    test) run pytest_gpu 600 $PYT ;;
    bounds) CYAES_LIBRARY=$R/build/variants/bounds.so run pytest_bounds 600 $PYT ;;
    smoke) run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" ;;
    soak) CYAES_SWEEP_CASES=${SOAK:-2000} run sweep_soak 900 python -u -m pytest tests/test_gpu_sweep.py -m gpu -x -q --timeout 600 --timeout-method thread ;;
    bench) run bench 400 python bench.py ;;
    quickbench) run quickbench 300 python bench.py --steps 3 --warmup 1 --no-cpu ;;
    profile)
      (cd /tmp && run rocprof_stats 300 rocprofv3 --kernel-trace --stats -d "$O/rocprof" -o run --output-format csv \
        -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --packet-configs none --relay-stream 0 --e2e-gib 0 --traffic none) || exit $?
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && run pmc_$c 300 rocprofv3 --pmc $c -d "$O/pmc_$c" -o run --output-format csv \
          -- python3 "$R/bench.py" --config E --e-passes 2 --steps 1 --warmup 0 --no-cpu --no-verify --no-clock \
             --packet-configs none --relay-stream 0 --e2e-gib 0 --traffic none) || exit $?
      done ;;
    cfgtest) run pytest_config_e 400 python -u -m pytest tests/test_config_e.py -m gpu -x -v --timeout 150 --timeout-method thread ;;
    pytest:*)  # pytest:FILE[::TEST] -- one test file or test, -m gpu
      A=${step#pytest:}
      T=pytest_$(basename "${A%%::*}" .py)
      run $T 400 python -u -m pytest "tests/$A" -m gpu -x -v --timeout 150 --timeout-method thread ;;
    batchertest) run pytest_batcher 300 python -u -m pytest tests/test_batcher.py -m gpu -x -v --timeout 150 --timeout-method thread ;;
    batcher)  # SEAL / OPEN host to host: zero-copy pools (pointer and offset submits), then the bounce path
      : > "$O/bench_batcher.jsonl"
      for cfg in "seal --pool 1" "seal --submit pooled" "open --pool 1" "open --submit pooled" "seal --pool 0" "open --pool 0"; do
        run bench_batcher_one 120 build/bench_batcher --op $cfg --threads 8 --window 8192 --seconds 4 ${BB_ARGS:-}
        grep '^{' "$O/bench_batcher_one.txt" >> "$O/bench_batcher.jsonl"
      done ;;
    hostlink) run hostlink 240 build/hostlink ;;
    bbprof:*)  # rocprofv3 kernel stats of one bench_batcher run (ARGS comma-separated)
      A=${step#bbprof:}
      T=bbprof_$(echo "$A" | tr -c 'a-z0-9' '_')
      (cd /tmp && run $T 180 rocprofv3 --kernel-trace --stats -d "$O/$T" -o run --output-format csv \
        -- "$R/build/bench_batcher" ${A//,/ } --threads 8 --seconds 2) || exit $?
      # keep the per-dispatch trace small: the first 20k dispatches
      f=$(find "$O/$T" -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && head -20000 "$f" > "$O/$T/trace_head.csv" && rm -f "$f" ;;
    bb:*)  # one bench_batcher run, arguments comma-separated: bb:--op,seal,--window,16384
      A=${step#bb:}
      CYAES_BATCHER_PROFILE=1 run bench_batcher_one 120 build/bench_batcher ${A//,/ } --threads ${BB_THREADS:-8} --seconds ${BB_SECONDS:-4}
      { grep '^{' "$O/bench_batcher_one.txt" | tr -d '\n'; echo -n ', '; grep '^\[cyaes_batcher\]' "$O/bench_batcher_one.txt" || echo; } >> "$O/bb.txt" ;;
    ab:*)
      IFS=: read -r _ A B ARGS <<< "$step"
      L="build/variants/$A.so build/variants/$B.so"
      RL="build/variants/$B.so build/variants/$A.so"
      T=$(echo "$ARGS" | tr -c 'A-Za-z0-9' '_')
      run ab_${A}_vs_${B}_$T 300 python tools/ab.py $L ${ARGS//,/ }
      run ab_${B}_vs_${A}_$T 300 python tools/ab.py $RL ${ARGS//,/ } ;;
    abenv:*)  # abenv:NAME=V[+NAME=V]:ARGS -- the product library against itself with those context settings
      IFS=: read -r _ ENVS ARGS <<< "$step"
      L="cyclone_amd/libcyaes.so cyclone_amd/libcyaes.so:${ENVS//+/:}"
      RL="cyclone_amd/libcyaes.so:${ENVS//+/:} cyclone_amd/libcyaes.so"
      T=abenv_$(echo "$ENVS$ARGS" | tr -c 'A-Za-z0-9' '_')
      run ${T} 300 python tools/ab.py $L ${ARGS//,/ }
      run ${T}_rev 300 python tools/ab.py $RL ${ARGS//,/ } ;;
    abrelay:*)
      IFS=: read -r _ A B <<< "$step"
      run abrelay_${A}_vs_${B} 300 python tools/ab_relay_layout.py --lib build/variants/$A.so build/variants/$B.so ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu] done"
