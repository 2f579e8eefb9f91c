#!/bin/bash
# Diagnostic: every LDS-DMA variant on the small transition convs of D-22 (batch 8).
cd ${GRAFT_REPO_ROOT:-.}
for o in "l4.0ds" "l4.0c1"; do
  ONLY="$o" TILES=4,6,7,8,9,10,12,13,15 timeout -k 10 200 python -u scripts/conv_micro.py 8 || exit 1
done
