#!/bin/bash
# Effective clock and MFMA-pipe utilisation per kernel of the bench workload (MI355X_MICROARCH.md
# 'DVFS give-back'): one PMC pass GRBM_GUI_ACTIVE + SQ_VALU_MFMA_BUSY_CYCLES with the kernel trace.
# usage (GPU box): bash scripts/pmc_clock.sh OUTNAME [bench args...]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES \
  --output-format csv -d $OUT/clk -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact-mode "$@" \
  > $OUT/clk.log 2>&1) || { echo "pmc pass failed"; tail -5 $OUT/clk.log; exit 1; }
python3 $R/scripts/pmc_clock.py $OUT/clk > $OUT/clock.json && cat $OUT/clock.json
