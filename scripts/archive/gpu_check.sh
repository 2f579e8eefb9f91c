#!/bin/bash
# Run on the GPU box (via gpurun): GPU tests, then a rocprofv3 kernel-trace of a short bench.
# usage: bash scripts/gpu_check.sh OUTNAME [bench args...]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
timeout -k 10 400 python -m pytest $R/tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
tail -3 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $OUT/bench.log 2>&1
echo "prof rc=$?"
