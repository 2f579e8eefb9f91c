#!/bin/bash
# Interleaved runs of one script per library build: bash scripts/lib_ab.sh OUT SCRIPT lib1 lib2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; SCRIPT=$2; shift 2
mkdir -p $OUT
for rep in 1 2 3; do for lib in "$@"; do
  echo "== $lib $(DRNMI_LIB=$R/video-seg-model-compress_amd/drnmi/$lib.so timeout -k 5 120 python $R/$SCRIPT 2>&1 | grep -v amdgpu.ids)" >> $OUT/ab.txt || exit 1
done; done
cat $OUT/ab.txt
