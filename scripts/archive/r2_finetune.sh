#!/bin/bash
# Fine-tune bench (config C4, D-54 + RMB 75 %, 1 GPU) plus its rocprofv3 kernel-trace summary.
# usage: bash scripts/r2_finetune.sh OUTNAME
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
timeout -k 10 400 python -u $R/bench_finetune.py --cpu-seconds 15 > $OUT/finetune.json 2> $OUT/finetune.err || { echo finetune failed; tail -5 $OUT/finetune.err; exit 1; }
cat $OUT/finetune.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ft_trace -o run --output-format csv -- \
  python3 $R/bench_finetune.py --no-cpu-baseline > $OUT/finetune_under_rocprof.log 2>&1) || { echo "trace failed"; exit 1; }
find $OUT/ft_trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/finetune_kernel_stats.csv
head -12 $OUT/finetune_kernel_stats.csv
