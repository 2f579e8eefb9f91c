#!/bin/bash
# 16x16 block-sparsity bound (diagnostic): conv_stag with the MFMAs of 2 of every wave's 8 16-row
# blocks removed (DRNMI_STAG_ABL=8, the 25 % of 16 x 32 weight units a 50 % 16 x 16 BlockPruner
# mask leaves all-zero; abl16: a pseudo-random 25 % of the units per wave and substep) against the
# default build, on the layer5-8 shapes.  bash scripts/r5_abl8.sh OUT
set -u
cd ${GRAFT_REPO_ROOT:-.}
OUT=gpurun_out/$1; mkdir -p $OUT
D=$PWD/video-seg-model-compress_amd/drnmi
for rep in 1 2; do for lib in libdrnmi libdrnmi_abl8 libdrnmi_abl16; do
  echo "== $lib" >> $OUT/abl8_micro.txt
  DRNMI_LIB=$D/$lib.so TILES=19 ONLY=l timeout -k 10 150 python scripts/conv_micro.py 8 2>/dev/null | head -5 >> $OUT/abl8_micro.txt || exit 1
done; done
