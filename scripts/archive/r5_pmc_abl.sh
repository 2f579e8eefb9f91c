#!/bin/bash
# PMC per variant for the 16x16 sparsity bound (diagnostic): LDS instructions / LDS activity / MFMA
# busy / clock of conv_stag on the D-22 layer8 shape, default build vs the random 25 % MFMA-skip
# ablation (DRNMI_STAG_ABL=16).  usage (GPU box): bash scripts/r5_pmc_abl.sh OUTNAME
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
for lib in libdrnmi libdrnmi_abl16; do
  (cd /tmp && DRNMI_LIB=$R/video-seg-model-compress_amd/drnmi/$lib.so ONLY=l8 TILES=19 timeout -k 10 120 rocprofv3 \
    --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/$lib -o run -- python3 $R/scripts/conv_micro.py 8 > $OUT/$lib.log 2>&1) || { echo "pmc $lib failed"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for lib in ("libdrnmi", "libdrnmi_abl16"):
    f = glob.glob(f"{out}/{lib}/**/run_counter_collection.csv", recursive=True)
    if not f:
        print(lib, "no counters"); continue
    acc = collections.defaultdict(float); n = collections.Counter(); dur = 0.0
    for r in csv.DictReader(open(f[0])):
        if "conv_stag_kernel" not in r.get("Kernel_Name", ""):
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
    d = {k: acc[k] / max(1, n[k]) for k in acc}
    gui = d.get("GRBM_GUI_ACTIVE", 0.0)
    print(lib, {k: f"{v:.4g}" for k, v in sorted(d.items())},
          "mfma_busy=%.3f" % (d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui / 8 * 1024) if gui else 0))
PY
