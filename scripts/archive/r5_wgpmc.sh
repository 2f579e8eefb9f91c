#!/bin/bash
# Diagnostic: wgrad micro timings + two SQ PMC passes over it: bash scripts/r5_wgpmc.sh OUT
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
timeout -k 10 120 python3 -u $R/scripts/wgrad_micro.py > $OUT/micro.log 2>&1 || { tail -5 $OUT/micro.log; exit 1; }
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/scripts/wgrad_micro.py > $OUT/p$i.log 2>&1) || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
  python3 $R/scripts/pmc_dump.py $OUT/p$i > $OUT/pmc$i.txt
  rm -rf $OUT/p$i
done
echo done
