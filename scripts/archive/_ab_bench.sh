#!/bin/bash
# A/B: bench lines of the default library and variants (diagnostic): bash scripts/_ab_bench.sh OUT FILTER lib...
cd ${GRAFT_REPO_ROOT:-.}
OUT=gpurun_out/$1; F=$2; shift 2; mkdir -p $OUT
for rep in 1 2; do
for lib in libdrnmi "$@"; do
  DRNMI_LIB=$PWD/video-seg-model-compress_amd/drnmi/$lib.so timeout -k 10 200 python -u bench.py --no-cpu-baseline > $OUT/$lib.$rep.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/$lib.$rep.json').read().strip().splitlines()[-1]); k=d['kernels']
print('$lib', round(d['value'],1), {n: v['avg_us'] for n, v in k.items() if '$F' in n})"
done
done
