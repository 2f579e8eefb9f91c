#!/bin/bash
# Round profile set (GPU box): GPU test suite, kernel-trace stats of the default bench and of the
# int8 / fp32x / fp32 benches, PMC HBM-traffic passes for all four.  usage: bash scripts/profile_round.sh OUTNAME
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest $R/tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/pytest_gpu.log; tail -3 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_bf16 -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-exact-mode > $OUT/bench_bf16_under_rocprof.log 2>&1) || { echo "trace bf16 failed"; exit 1; }
for P in int8 fp32x fp32; do
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$P -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-exact-mode --precision $P > $OUT/bench_${P}_under_rocprof.log 2>&1) || { echo "trace $P failed"; exit 1; }
done
bash $R/scripts/pmc_traffic.sh $1/pmc_bf16 > /dev/null || exit 1
bash $R/scripts/pmc_mfma.sh $1/mfma_bf16 || exit 1
for P in int8 fp32x fp32; do
bash $R/scripts/pmc_traffic.sh $1/pmc_$P --precision $P > /dev/null || exit 1
bash $R/scripts/pmc_mfma.sh $1/mfma_$P --precision $P || exit 1
done
echo done
