#!/bin/bash
# Diagnostic: halo micro on the shipped library and the ablation builds (scripts/build_variant_src.sh)
cd ${GRAFT_REPO_ROOT:-.}
echo "== base"; timeout -k 5 120 python scripts/halo_micro.py 17 18 || exit 1
echo "== base RES=0"; RES=0 timeout -k 5 120 python scripts/halo_micro.py 17 18 || exit 1
for v in "$@"; do
  echo "== rw$v"
  DRNMI_LIB=$PWD/video-seg-model-compress_amd/drnmi/libdrnmi_rw$v.so RES=0 timeout -k 5 120 python scripts/halo_micro.py 18 || exit 1
done
