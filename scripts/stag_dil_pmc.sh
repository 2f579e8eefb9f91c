#!/bin/bash
# conv_stag at dilation 1 vs 4 (no residual, batch 4, D-22 layer8 / layer6 shapes): SQ cycle
# counters + the clock (GRBM_GUI_ACTIVE) and the L2 hit counters, one rocprofv3 --pmc pass each,
# every pass its own process per shape.  usage (GPU box): bash scripts/stag_dil_pmc.sh OUTNAME
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="TCC_HIT_sum TCC_MISS_sum"
i=0
for shape in "l8 512x512 d1" "l6 512x512 d4 nores" "l7 512x512 d2"; do
  for pass in A B; do
    ctrs=${!pass}
    (cd /tmp && ONLY="$shape" TILES=19 timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/s$i$pass -o run -- \
      python3 $R/scripts/conv_micro.py 4 > $OUT/s$i$pass.log 2>&1) || { echo "pass $shape $pass failed"; exit 1; }
  done
  i=$((i+1))
done
echo done
