#!/bin/bash
# A/B of the default library against variants on the residual shapes (conv_micro) and the
# bench line (diagnostic): bash scripts/r5_ab.sh OUT lib...
set -u
cd ${GRAFT_REPO_ROOT:-.}
OUT=gpurun_out/$1; shift; mkdir -p $OUT
D=$PWD/video-seg-model-compress_amd/drnmi
for rep in 1 2; do for lib in libdrnmi "$@"; do
  echo "== $lib" >> $OUT/micro.txt
  DRNMI_LIB=$D/$lib.so TILES=17,19 timeout -k 10 150 python scripts/conv_micro.py 8 >> $OUT/micro.txt 2>/dev/null || exit 1
done; done
for rep in 1 2; do for lib in libdrnmi "$@"; do
  DRNMI_LIB=$D/$lib.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-exact-mode > $OUT/$lib.$rep.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/$lib.$rep.json').read().strip().splitlines()[-1]); k=d['kernels']
print('$lib', round(d['value'],1), {n: v['avg_us'] for n, v in k.items()})" >> $OUT/bench.txt
done; done
