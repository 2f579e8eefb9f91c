#!/bin/bash
# C3 block-sparse A/B (dense vs K-step compaction) on D-38, bf16: usage bash scripts/r2_c3.sh OUTNAME [BHxBW]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
BLK=${2:-256x64}
mkdir -p $OUT
for mode in dense sparse dense sparse; do
  extra=""; [ $mode = sparse ] && extra="--block-sparse"
  timeout -k 10 300 python -u $R/bench.py --arch drn_d_38 --prune block:$BLK:0.5 $extra --no-cpu-baseline --steps 10 --warmup 3 \
    > $OUT/c3_${BLK}_$mode.json 2> $OUT/c3_${BLK}_$mode.err || { echo "c3 $mode failed"; tail -5 $OUT/c3_${BLK}_$mode.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c3_${BLK}_$mode.json')); print('$mode', round(d['value'],1), d['config'].get('block_sparse'))"
done
