#!/bin/bash
# conv_stag ablations (diagnostic builds): 1 no in-loop DMA, 2 no MFMA, 4 no fragment reads
set -u
cd ${GRAFT_REPO_ROOT:-.}
D=$PWD/video-seg-model-compress_amd/drnmi
for rep in 1 2; do for lib in libdrnmi libdrnmi_abl1 libdrnmi_abl2 libdrnmi_abl3 libdrnmi_abl4 libdrnmi_abl6 libdrnmi_abl7; do
  echo "== $lib"; DRNMI_LIB=$D/$lib.so TILES=19 ONLY=l timeout -k 10 120 python scripts/conv_micro.py 8 2>/dev/null | head -5 || exit 1
done; done
