#!/bin/bash
# PMC WRITE_SIZE/FETCH_SIZE for a libcyaes variant via tools/ab.py (one lib per run).
# usage: scripts/ab_pmc.sh OUTDIR lib.so [lib2.so ...]
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/$1; shift
export TMPDIR=/tmp; mkdir -p "$OUT"; cd /tmp || exit 1
for lib in "$@"; do
  n=$(basename "$lib" .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -d "$OUT/$n.$c" -o run --output-format csv -- python3 "$R/tools/ab.py" "$R/$lib" --rounds 1 > "$OUT/$n.$c.log" 2>&1
    rc=$?; echo "[pmc] $n $c rc=$rc"
    if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  done
done
