#!/bin/bash
# Run a subset of GPU tests on the box: bash scripts/gpu_tests.sh OUTNAME [pytest args...]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
tail -25 $OUT/pytest.log
exit $rc
