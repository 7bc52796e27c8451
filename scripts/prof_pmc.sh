#!/bin/bash
# PMC passes over bench.py (GPU box).  Each pass is its own rocprofv3 run with
# --pmc only (no trace domains besides kernel dispatch), per the pool rules.
# usage: scripts/prof_pmc.sh OUTDIR "bench args" "COUNTERS;COUNTERS;..."
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/$1; ARGS=$2; PASSES=$3
export TMPDIR=/tmp
mkdir -p "$OUT"
cd /tmp || exit 1
i=0
IFS=';' read -ra P <<< "$PASSES"
for pass in "${P[@]}"; do
  i=$((i+1))
  echo "[prof] pass $i: $pass"
  timeout -k 10 300 rocprofv3 --pmc $pass -d "$OUT/pass$i" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "[prof] pass $i rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "[prof] stopping"; exit $rc; fi
done
