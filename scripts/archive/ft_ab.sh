#!/bin/bash
# fp32x fine-tune (C4) A/B, interleaved (GPU box).  Each variant: "LIB[:ENV=V,...]" (LIB under drnmi/).
# usage: bash scripts/ft_ab.sh OUT variant1 variant2 ...   e.g. libdrnmi libdrnmi:DRNMI_BATCHED_PACK=0
set -u
cd ${GRAFT_REPO_ROOT:-.}
OUT=gpurun_out/$1; shift; mkdir -p $OUT
D=$PWD/video-seg-model-compress_amd/drnmi
for rep in 1 2; do for v in "$@"; do
  lib=${v%%:*}; envs=""; [ "$v" != "$lib" ] && envs=$(echo ${v#*:} | tr ',' ' ')
  tag=$(echo $v | tr ':=,' '___')
  env DRNMI_LIB=$D/$lib.so $envs timeout -k 10 200 python -u bench_finetune.py --precision fp32x --no-cpu-baseline \
    --steps 6 --warmup 2 > $OUT/ft_$tag.$rep.json 2>$OUT/ft_$tag.$rep.err || { tail -5 $OUT/ft_$tag.$rep.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/ft_$tag.$rep.json').read().strip().splitlines()[-1]); print('$v', round(d['value'],2), round(d['ms_per_step'],2))" >> $OUT/ft_ab.txt
done; done
cat $OUT/ft_ab.txt
