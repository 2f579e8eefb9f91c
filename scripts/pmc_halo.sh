#!/bin/bash
# Diagnostic: one PMC pass (+ kernel trace) over scripts/halo_micro.py; usage: bash scripts/pmc_halo.sh OUT [tiles]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
(cd /tmp && timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS \
  --output-format csv -d $OUT/p -o run -- python3 $R/scripts/halo_micro.py "$@" > $OUT/p.log 2>&1) || { echo "pmc pass failed"; tail -5 $OUT/p.log; exit 1; }
python3 $R/scripts/pmc_dump.py $OUT/p
