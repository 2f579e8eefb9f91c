#!/bin/bash
# A/B bench lines (diagnostic): bash scripts/r5_ab2.sh OUT "bench args" lib...
set -u
cd ${GRAFT_REPO_ROOT:-.}
OUT=gpurun_out/$1; ARGS=$2; shift 2; mkdir -p $OUT
D=$PWD/video-seg-model-compress_amd/drnmi
tag=$(echo "$ARGS" | tr -c 'a-z0-9' '_')
for rep in 1 2; do for lib in libdrnmi "$@"; do
  DRNMI_LIB=$D/$lib.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-exact-mode $ARGS > $OUT/$lib.$tag.$rep.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/$lib.$tag.$rep.json').read().strip().splitlines()[-1]); k=d['kernels']
print('$lib', '$ARGS', round(d['value'],1), {n: v['avg_us'] for n, v in k.items()})" >> $OUT/bench.txt
done; done
