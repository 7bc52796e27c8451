#!/bin/bash
# r02: VALU / LDS utilisation of the ragged kernels against the uniform ones on
# the same 1 M x 1,472-B payloads (tools/ab_ragged.py), one --pmc run per pass.
# usage: scripts/pmc_ragged.sh OUTDIR
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/$1
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp || exit 1
P1="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_ANY GRBM_GUI_ACTIVE"
run() {  # run NAME COUNTERS
  local name=$1 ctr=$2
  echo "[pmc] $name"
  timeout -s KILL 200 rocprofv3 --pmc $ctr -d "$O/$name" -o run --output-format csv -- python3 "$R/tools/ab_ragged.py" --rounds 2 --sizes 1048576:1472 > "$O/$name.log" 2>&1
  local rc=$?
  echo "[pmc] $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$O/$name.log"; exit $rc; fi
}
run p1 "$P1"
run p2 "$P2"
run p3 "$P3"
echo "[pmc] done"
