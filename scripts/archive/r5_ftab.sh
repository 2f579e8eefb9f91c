#!/bin/bash
# fp32x fine-tune A/B of the default library against variants (diagnostic): bash scripts/r5_ftab.sh OUT lib...
set -u
cd ${GRAFT_REPO_ROOT:-.}
OUT=gpurun_out/$1; shift; mkdir -p $OUT
D=$PWD/video-seg-model-compress_amd/drnmi
for rep in 1 2; do for lib in libdrnmi "$@"; do
  DRNMI_LIB=$D/$lib.so timeout -k 10 200 python -u bench_finetune.py --precision fp32x --no-cpu-baseline --steps 6 --warmup 2 > $OUT/ft_$lib.$rep.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/ft_$lib.$rep.json').read().strip().splitlines()[-1]); print('$lib', round(d['value'],2), round(d['ms_per_step'],2))" >> $OUT/ft_ab.txt
done; done
