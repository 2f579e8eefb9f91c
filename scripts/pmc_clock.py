"""Per-kernel effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration) and MFMA-pipe utilisation
(SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs)) from scripts/pmc_clock.sh output."""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        name = r["Kernel_Name"].replace("void ", "", 1).replace("drnmi::(anonymous namespace)::", "")
        if name.endswith(")") and "(" in name:
            name = name[:name.rfind("(")]
        key = (name, r.get("Dispatch_Id") or r.get("Correlation_Id"))
        acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
        for k in ("Start_Timestamp", "End_Timestamp"):
            if k in r:
                acc[key][k] = float(r[k])
per = collections.defaultdict(lambda: collections.defaultdict(float))
for (name, _), v in acc.items():
    if "End_Timestamp" not in v:
        continue
    dur = (v["End_Timestamp"] - v["Start_Timestamp"]) * 1e-9
    if dur <= 0:
        continue
    per[name]["dur"] += dur
    per[name]["grbm"] += v.get("GRBM_GUI_ACTIVE", 0.0)
    per[name]["mfma"] += v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    per[name]["n"] += 1
out = {}
for name, v in sorted(per.items(), key=lambda kv: -kv[1]["dur"]):
    cyc = v["grbm"] / 8.0
    out[name] = {"launches": int(v["n"]), "avg_us": round(v["dur"] / v["n"] * 1e6, 1),
                 "eff_clock_ghz": round(cyc / v["dur"] / 1e9, 3),
                 "mfma_busy_frac": round(v["mfma"] / (cyc * 1024), 4) if cyc else None}
json.dump(out, sys.stdout, indent=1)
