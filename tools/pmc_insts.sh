#!/bin/bash
# PMC instruction and LDS counters per relay-layout launch (rocprofv3 --pmc, two
# passes per layout; tools/pmc_summary.py DIR... --match k_decrypt_flat).
# usage: tools/pmc_insts.sh OUT_SUBDIR LAYOUT[,LAYOUT...] [ab_relay_layout.py args...]
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
LAYOUTS=$2; shift 2
cd /tmp; export TMPDIR=/tmp
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
for ly in ${LAYOUTS//,/ }; do
  i=0
  for p in "$P1" "$P2"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $p -d $O/${ly}_p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ab_relay_layout.py --api strided --rounds 3 --layouts $ly "$@" > $O/${ly}_p$i.log 2>&1
  done
done
