#!/bin/bash
# conv_x6 A/B (GPU box): interleaved x6_micro runs per library (time + output SHA-1).
# usage: bash scripts/x6_ab.sh OUT lib1 lib2 ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib" >> $OUT/x6_micro.txt
    DRNMI_LIB=$R/video-seg-model-compress_amd/drnmi/$lib.so timeout -k 5 200 python $R/scripts/x6_micro.py 2>&1 | grep -v amdgpu.ids >> $OUT/x6_micro.txt || exit 1
  done
done
cat $OUT/x6_micro.txt
