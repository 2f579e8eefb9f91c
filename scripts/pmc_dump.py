"""Per-kernel average of every collected PMC counter per dispatch, plus the derived clock
(GRBM_GUI_ACTIVE / 8 XCDs / duration) and MFMA busy fraction (SQ_VALU_MFMA_BUSY_CYCLES /
(clock cycles x 1024 SIMDs)).  python scripts/pmc_dump.py <rocprofv3 -d dir>"""
import collections
import csv
import glob
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{sys.argv[1]}/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("void ", "", 1).replace("drnmi::(anonymous namespace)::", "")
        name = name[:name.rfind("(")] if name.endswith(")") and "(" in name else name
        key = (name, r.get("Dispatch_Id") or r.get("Correlation_Id"))
        acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
        for k in ("Start_Timestamp", "End_Timestamp"):
            if k in r:
                acc[key][k] = float(r[k])
per = collections.defaultdict(lambda: collections.defaultdict(list))
for (name, _), v in acc.items():
    for k, x in v.items():
        per[name][k].append(x)
    if "End_Timestamp" in v:
        per[name]["dur_us"].append((v["End_Timestamp"] - v["Start_Timestamp"]) * 1e-3)
for name, d in per.items():
    if not name.startswith(("conv", "stem", "patch", "up8", "wgrad")):
        continue
    avg = {k: sum(x) / len(x) for k, x in d.items() if k not in ("Start_Timestamp", "End_Timestamp")}
    line = f"{name[:60]:60s} n={len(d.get('dur_us', [0]))}"
    for k, x in sorted(avg.items()):
        line += f" {k}={x:.4g}"
    if "GRBM_GUI_ACTIVE" in avg and avg.get("dur_us"):
        ghz = avg["GRBM_GUI_ACTIVE"] / 8 / (avg["dur_us"] * 1e3)
        line += f" clock_GHz={ghz:.3f}"
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
            line += f" mfma_busy={avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (avg['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}"
    print(line)
