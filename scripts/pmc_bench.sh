#!/bin/bash
# Diagnostic: one PMC pass (+ kernel trace) over a short bench run; per-kernel averages.
# usage: bash scripts/pmc_bench.sh OUT "COUNTERS" [bench args]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; CNT=$2; shift 2
mkdir -p $OUT
(cd /tmp && timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --pmc $CNT --output-format csv -d $OUT/p -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exact-mode "$@" > $OUT/p.log 2>&1) || { echo "pmc pass failed"; tail -5 $OUT/p.log; exit 1; }
python3 $R/scripts/pmc_dump.py $OUT/p
