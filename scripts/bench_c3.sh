#!/bin/bash
# C2 default + C3 (D-38 + BlockPruner 50%) dense vs unit-skipping, on the GPU box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err || exit 1
for spec in block:16x16:0.5 block:16x32:0.5; do
  tag=$(echo $spec | tr ':' '_')
  timeout -k 10 300 python $R/bench.py --arch drn_d_38 --prune $spec --block-sparse --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c3_${tag}_sparse.json 2> $OUT/c3_${tag}_sparse.err || exit 1
  timeout -k 10 300 python $R/bench.py --arch drn_d_38 --prune $spec --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c3_${tag}_dense.json 2> $OUT/c3_${tag}_dense.err || exit 1
done
for f in $OUT/*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], round(d['value'],1), d['roofline']['kernel'], d['roofline']['achieved'], d['config'].get('block_sparse'))"; done
