#!/bin/bash
# stem+layer1 fused kernel ablations (diagnostic builds): which part bounds it
set -u
cd ${GRAFT_REPO_ROOT:-.}
D=$PWD/video-seg-model-compress_amd/drnmi
for rep in 1 2; do for lib in libdrnmi libdrnmi_nolut libdrnmi_nostem libdrnmi_nol1 libdrnmi_nost libdrnmi_nomfma libdrnmi_skel; do
  echo "== $lib $(DRNMI_LIB=$D/$lib.so ONLY=stem+ timeout -k 10 120 python scripts/patch_micro.py 8 2>/dev/null)" || exit 1
done; done
