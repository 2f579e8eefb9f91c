#!/bin/bash
# A/B of front-kernel builds: bash scripts/front_ab.sh lib1 lib2 ...  (names under drnmi/, "" = default)
cd ${GRAFT_REPO_ROOT:-.}
for rep in 1 2; do
for lib in "$@"; do
  echo "== $lib"
  DRNMI_LIB=$PWD/video-seg-model-compress_amd/drnmi/$lib.so CMP=0 timeout -k 5 120 python scripts/front_micro.py || exit 1
done
done
