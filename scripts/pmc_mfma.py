"""Per-kernel MFMA-pipe utilisation and held clock of the bench workload, from scripts/pmc_mfma.sh.

One rocprofv3 pass with GRBM_GUI_ACTIVE + SQ_VALU_MFMA_BUSY_CYCLES (kernel trace on, no other
tracing).  Normalisation (MI355X_MICROARCH.md 'DVFS give-back' and the SQ PMC units row):
  clock cycles of a dispatch  = GRBM_GUI_ACTIVE / 8      (rocprofv3 sums the 8 XCDs)
  mfma_busy                   = SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs)
  eff_clock_ghz               = clock cycles / dispatch duration
`step` aggregates every dispatch of the timed steps (sum of busy over sum of SIMD-cycles): the
MFMA utilisation of the whole seg_video step, not only of its dominant kernel.

usage: pmc_mfma.py OUT ARCH HEIGHT WIDTH FRAMES PRECISION "COMMAND" > json"""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
config = {"arch": sys.argv[2], "height": int(sys.argv[3]), "width": int(sys.argv[4]),
          "frames_per_gpu_step": int(sys.argv[5]), "precision": sys.argv[6]}
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("void ", "", 1).replace("drnmi::(anonymous namespace)::", "")
        if name.endswith(")") and "(" in name:
            name = name[:name.rfind("(")]
        key = (name, r.get("Dispatch_Id") or r.get("Correlation_Id"))
        acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
        for k in ("Start_Timestamp", "End_Timestamp"):
            if k in r:
                acc[key][k] = float(r[k])
per = collections.defaultdict(lambda: collections.defaultdict(float))
tot = collections.defaultdict(float)
for (name, _), v in acc.items():
    if "End_Timestamp" not in v:
        continue
    dur = (v["End_Timestamp"] - v["Start_Timestamp"]) * 1e-9
    if dur <= 0:
        continue
    cyc = v.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    mf = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    for d in (per[name], tot):
        d["dur"] += dur
        d["cyc"] += cyc
        d["mfma"] += mf
        d["n"] += 1


def row(v):
    return {"launches": int(v["n"]), "avg_us": round(v["dur"] / v["n"] * 1e6, 1),
            "eff_clock_ghz": round(v["cyc"] / v["dur"] / 1e9, 3),
            "mfma_busy": round(v["mfma"] / (v["cyc"] * 1024), 4) if v["cyc"] else None}


kernels = {k: row(v) for k, v in sorted(per.items(), key=lambda kv: -kv[1]["dur"])}
json.dump({"config": config, "command": sys.argv[7] if len(sys.argv) > 7 else "scripts/pmc_mfma.sh",
           "normalisation": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / ((GRBM_GUI_ACTIVE / 8 XCDs) x 1024 SIMDs) "
                            "per dispatch, averaged over the kernel's dispatches by cycle weight; eff_clock = "
                            "(GRBM_GUI_ACTIVE / 8) / dispatch duration; 'all_dispatches' pools every dispatch of "
                            "the run (the whole seg_video step)",
           "all_dispatches": row(tot) if tot else None, "kernels": kernels}, sys.stdout, indent=1)
