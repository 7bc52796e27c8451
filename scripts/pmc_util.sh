#!/bin/bash
# VALU / LDS utilisation counters (GPU box), one rocprofv3 --pmc run per pass:
# the T-table kernels (bench.py config C) and the bitsliced prototype.
# usage: scripts/pmc_util.sh OUTDIR
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/$1
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp || exit 1
P1="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
run() {  # run NAME COUNTERS CMD...
  local name=$1 ctr=$2; shift 2
  echo "[pmc] $name"
  timeout -s KILL 200 rocprofv3 --pmc $ctr -d "$O/$name" -o run --output-format csv -- "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[pmc] $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$O/$name.log"; exit $rc; fi
}
run tt_p1 "$P1" python3 "$R/bench.py" --config C --steps 2 --warmup 0 --no-cpu --no-verify --no-clock --packet-configs none
run tt_p2 "$P2" python3 "$R/bench.py" --config C --steps 2 --warmup 0 --no-cpu --no-verify --no-clock --packet-configs none
run bs_p1 "$P1" "$R/build/bitslice" 65536 2 16
echo "[pmc] done"
