#!/bin/bash
# conv_stag tile-deal / cache-policy A/B (GPU box): interleaved timings of the layer5-8 shapes at
# batch 8 per library, then per library PMC passes over the l8 shape (HBM fetch/write bytes,
# clock + MFMA busy, L2 hit/miss).  usage: bash scripts/stag_map_ab.sh OUTNAME lib1 lib2 ...
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib" >> $OUT/micro.txt
    DRNMI_LIB=$R/video-seg-model-compress_amd/drnmi/$lib.so TILES=19 ONLY=l timeout -k 5 200 python $R/scripts/conv_micro.py 8 >> $OUT/micro.txt 2>&1 || exit 1
  done
done
export ONLY="l8" TILES=19
for lib in "$@"; do
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    (cd /tmp && DRNMI_LIB=$R/video-seg-model-compress_amd/drnmi/$lib.so timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/$lib/pmc$i -o run -- python3 $R/scripts/conv_micro.py 8 > $OUT/$lib.pmc$i.log 2>&1) || { echo "pmc $lib $i failed"; exit 1; }
  done
  echo "== $lib" >> $OUT/pmc_summary.txt
  python3 $R/scripts/pmc_table.py $OUT/$lib conv_stag >> $OUT/pmc_summary.txt
done
cat $OUT/micro.txt $OUT/pmc_summary.txt
