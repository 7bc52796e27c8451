#!/bin/bash
# LDS / VALU utilisation counters for config B (1 M x 1,472 B) vs C, one --pmc run per pass.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/$1
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp || exit 1
P1="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
for cfg in B C; do
  echo "[pmc] $cfg"
  timeout -s KILL 200 rocprofv3 --pmc $P1 -d "$O/$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 4 --warmup 1 --no-cpu --no-verify --no-clock --packet-configs none > "$O/$cfg.log" 2>&1
  rc=$?; echo "[pmc] $cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
echo done
