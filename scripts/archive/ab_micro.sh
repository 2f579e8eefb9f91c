#!/bin/bash
# A/B of conv_big builds on the micro shapes: bash scripts/ab_micro.sh lib1 lib2 ...  (names under drnmi/)
cd ${GRAFT_REPO_ROOT:-.}
for rep in 1 2; do
for lib in "$@"; do
  echo "== $lib"
  DRNMI_LIB=$PWD/video-seg-model-compress_amd/drnmi/$lib.so TILES=${TILES:-5} ONLY=${ONLY:-l} timeout -k 5 200 python scripts/conv_micro.py 8 || exit 1
done
done
