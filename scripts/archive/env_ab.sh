#!/bin/bash
# Interleaved bench A/B of an environment switch on one box: bash scripts/env_ab.sh OUT VAR "v1 v2 ..." [bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; VAR=$2; VALS=$3; shift 3
mkdir -p $OUT
for rep in 1 2; do
for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python -u $R/bench.py --no-cpu-baseline --no-exact-mode "$@" > $OUT/b_${v}_$rep.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/b_${v}_$rep.json').read().strip().splitlines()[-1])
print('$VAR=$v', round(d['value'],1), round(d['ms_per_step'],3), d['network_roofline']['frac'])" >> $OUT/ab.txt
done; done
cat $OUT/ab.txt
