#!/bin/bash
# seg conv variant A/B inside the bench (per-kernel table)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r6_segab; mkdir -p $OUT
for rep in 1 2; do
for v in -1 8 9 3; do
  DRNMI_SEG_VARIANT=$v timeout -k 10 200 python -u $R/bench.py --no-cpu-baseline --no-exact-mode --steps 10 > $OUT/b_$v.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/b_$v.json').read().strip().splitlines()[-1])
print('$v', round(d['value'],1), {k: v['avg_us'] for k, v in d['kernels'].items() if 'stag' not in k and 'front' not in k and 'block' not in k})" >> $OUT/ab.txt
done; done
cat $OUT/ab.txt
