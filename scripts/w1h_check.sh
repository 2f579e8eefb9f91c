#!/bin/bash
# conv_w1h (tile 23) bring-up: bit identity vs conv_stag128 / conv_stag (tile 19) and conv_w1
# (tile 22) after the geometry template, then the interleaved micro on the layer4-8 shapes at
# batch 8.  usage (GPU box): bash scripts/w1h_check.sh OUTNAME
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
timeout -k 10 240 python -u -m pytest $R/tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "w1_kernel or w1h_kernel or stag_kernel_bit or stag128" > $O/pytest_w1h.log 2>&1
rc=$?; tail -3 $O/pytest_w1h.log; [ $rc -ne 0 ] && exit $rc
for s in l4 l5 l8 l6.0c1; do
  ONLY=$s TILES=19,22,23 timeout -k 10 120 python -u $R/scripts/conv_micro.py 8 >> $O/micro.log 2>&1 || exit 1
done
grep -v amdgpu.ids $O/micro.log
