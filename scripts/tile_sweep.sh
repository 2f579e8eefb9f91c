#!/bin/bash
# Every forced conv tile on the small transition convs of D-22 (batch 8; n/a = tile refuses the shape).
# usage (GPU box): bash scripts/tile_sweep.sh OUT
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p $OUT
for only in "l3.0c1" "l4.0c1" "l3 64" "l4 128" "seg"; do
  TILES=$(seq -s, 0 20) ONLY="$only" timeout -k 5 300 python $R/scripts/conv_micro.py 8 2>&1 | grep -v amdgpu.ids >> $OUT/tile_sweep.txt || exit 1
done
cat $OUT/tile_sweep.txt
