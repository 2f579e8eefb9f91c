#!/bin/bash
# Round-4 profile set (GPU box): rocprofv3 kernel-trace stats of the bf16 and fp32x benches, PMC
# HBM-traffic passes for both (separate FETCH_SIZE / WRITE_SIZE runs, kernel-trace only).
# usage: bash scripts/r4_profile.sh OUTNAME
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
for prec in bf16 fp32x int8; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$prec -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-exact-mode --precision $prec > $OUT/bench_${prec}_under_rocprof.log 2>&1) || { echo "trace $prec failed"; exit 1; }
  find $OUT/trace_$prec -name "run_kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/${prec}_kernel_stats.csv
  bash $R/scripts/pmc_traffic.sh $1/pmc_$prec --precision $prec > /dev/null || exit 1
  echo "$prec done"
done
head -4 $OUT/bf16_kernel_stats.csv
bash $R/scripts/pmc_bench.sh $1/pmc_sq "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS" > $OUT/pmc_sq.txt 2>&1 || exit 1
echo profile done
