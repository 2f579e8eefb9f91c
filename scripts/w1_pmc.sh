#!/bin/bash
# conv_w1 (tile 22) vs conv_stag (tile 19) on the D-22 layer8 shape at batch 8: SQ cycle counters
# + MFMA busy + clock, one rocprofv3 --pmc pass per tile.  usage (GPU box): bash scripts/w1_pmc.sh OUTNAME
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for t in 19 22; do
  (cd /tmp && ONLY="l8" TILES=$t timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $A --output-format csv -d $OUT/t$t -o run -- \
    python3 $R/scripts/conv_micro.py 8 > $OUT/t$t.log 2>&1) || { echo "pass $t failed"; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
for t in (19, 22):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for f in glob.glob(f"{sys.argv[1]}/t{t}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "conv_" not in k: continue
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            acc[(k, d)][r["Counter_Name"]] += float(r["Counter_Value"])
    tot = collections.defaultdict(float); cnt = 0
    for (k, d), v in acc.items():
        cnt += 1
        for c, x in v.items(): tot[c] += x
    v = {c: x / max(cnt, 1) for c, x in tot.items()}
    cyc = v.get("GRBM_GUI_ACTIVE", 0) / 8
    print(f"tile {t}: dispatches {cnt}  " + "  ".join(f"{c} {x:.4g}" for c, x in sorted(v.items())))
    if cyc:
        print(f"   mfma_busy {v.get('SQ_VALU_MFMA_BUSY_CYCLES',0)/(cyc*1024):.3f}  wait_any/wave {v.get('SQ_WAIT_ANY',0)/max(v.get('SQ_WAVE_CYCLES',1),1):.3f}  "
              f"wait_inst/wave {v.get('SQ_WAIT_INST_ANY',0)/max(v.get('SQ_WAVE_CYCLES',1),1):.3f}  active/wave {v.get('SQ_ACTIVE_INST_ANY',0)/max(v.get('SQ_WAVE_CYCLES',1),1):.3f}  "
              f"lds_active/clk {v.get('SQ_LDS_IDX_ACTIVE',0)/cyc:.3g}")
PY
