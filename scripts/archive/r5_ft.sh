#!/bin/bash
# fine-tune bench lines (fp32x, fp32) and the fp32x rocprofv3 kernel stats: bash scripts/r5_ft.sh OUT
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python -u $R/bench_finetune.py --precision fp32x --cpu-seconds 10 > $OUT/finetune_fp32x.json 2> $OUT/finetune_fp32x.err || { tail -5 $OUT/finetune_fp32x.err; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ft_trace -o run --output-format csv -- \
  python3 $R/bench_finetune.py --precision fp32x --no-cpu-baseline --steps 5 --warmup 2 > $OUT/finetune_under_rocprof.log 2>&1) || { echo "trace failed"; exit 1; }
find $OUT/ft_trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/finetune_fp32x_kernel_stats.csv
rm -rf $OUT/ft_trace
