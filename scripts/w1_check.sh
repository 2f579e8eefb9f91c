#!/bin/bash
# conv_w1 (tile 22) bring-up: bit identity vs conv_stag (tile 19), then the interleaved micro on the
# D-22 layer5-8 shapes at batch 8.  usage (GPU box): bash scripts/w1_check.sh OUTNAME
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
timeout -k 10 180 python -u -m pytest $R/tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "w1_kernel or stag_kernel_bit" > $O/pytest_w1.log 2>&1
rc=$?; tail -3 $O/pytest_w1.log; [ $rc -ne 0 ] && exit $rc
for s in l8 l7 l6 l5; do
  ONLY=$s TILES=19,22 timeout -k 10 120 python -u $R/scripts/conv_micro.py 8 >> $O/micro.log 2>&1 || exit 1
done
cat $O/micro.log
