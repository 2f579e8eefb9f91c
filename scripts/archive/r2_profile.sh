#!/bin/bash
# Round-2 profile set (GPU box): rocprofv3 kernel-trace stats of the bf16 and fp32x benches, PMC
# HBM-traffic passes for both (separate FETCH_SIZE / WRITE_SIZE runs, kernel-trace only).
# usage: bash scripts/r2_profile.sh OUTNAME
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
for prec in bf16 fp32x; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$prec -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --precision $prec > $OUT/bench_${prec}_under_rocprof.log 2>&1) || { echo "trace $prec failed"; exit 1; }
  find $OUT/trace_$prec -name "run_kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/${prec}_kernel_stats.csv
  bash $R/scripts/pmc_traffic.sh $1/pmc_$prec --precision $prec > /dev/null || exit 1
  echo "$prec done"
done
head -4 $OUT/bf16_kernel_stats.csv
