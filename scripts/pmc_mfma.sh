#!/bin/bash
# MFMA-pipe utilisation and held clock per kernel of the bench workload (north_star: "MFMA
# utilisation reported against MI355X peak"): one PMC pass GRBM_GUI_ACTIVE + SQ_VALU_MFMA_BUSY_CYCLES
# with the kernel trace, then scripts/pmc_mfma.py -> OUT/mfma.json (bench.py reads the committed
# copy, profiles/*_pmc_mfma.json, into roofline.mfma_busy).
# usage (GPU box): bash scripts/pmc_mfma.sh OUTNAME [bench args...]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES \
  --output-format csv -d $OUT/mfma -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline \
  --no-exact-mode "$@" > $OUT/mfma.log 2>&1) || { echo "pmc mfma pass failed"; tail -5 $OUT/mfma.log; exit 1; }
PREC=bf16
prev=""
for a in "$@"; do [ "$prev" = "--precision" ] && PREC=$a; prev=$a; done
python3 $R/scripts/pmc_mfma.py $OUT/mfma drn_d_22 1024 2048 8 $PREC \
  "scripts/pmc_mfma.sh: rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES over python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact-mode $*" \
  > $OUT/mfma.json && echo "mfma ok $PREC"
