"""Summarise scripts/pmc_cmd.sh output: mean counter value per kernel over its dispatches."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if filt not in k:
            continue
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    print(k[:110])
    # per dispatch mean (each dispatch appears once per counter, summed over dims already)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")
