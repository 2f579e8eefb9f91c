#!/bin/bash
# HBM traffic per kernel launch of the bench workload (MI355X_MICROARCH.md §HBM): two PMC
# passes (FETCH_SIZE, WRITE_SIZE cannot share one), then scripts/pmc_traffic.py.
# usage (GPU box): bash scripts/pmc_traffic.sh OUTNAME [bench args...]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact-mode "$@" > $OUT/$c.log 2>&1) || { echo "pass $c failed"; exit 1; }
done
# the workload's config (bench.py defaults unless --precision is given) for bench.py's lookup
PREC=bf16
prev=""
for a in "$@"; do [ "$prev" = "--precision" ] && PREC=$a; prev=$a; done
python3 $R/scripts/pmc_traffic.py $OUT drn_d_22 1024 2048 8 $PREC \
  "scripts/pmc_traffic.sh: rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE, over python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact-mode $*" \
  > $OUT/traffic.json && cat $OUT/traffic.json
