"""Per-kernel HBM bytes per launch from scripts/pmc_traffic.sh output.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KB) reports half the bytes of wide
coalesced reads -> x2; WRITE_SIZE (KB) is exact for 16-B-per-lane stores.  Infinity-Cache hits
are counted, so this is L2 <-> fabric traffic, an upper bound on HBM bytes."""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
# optional workload description (bench.py pmc_traffic matches "config" against its own run):
#   pmc_traffic.py OUT ARCH HEIGHT WIDTH FRAMES PRECISION "COMMAND"
config = None
if len(sys.argv) >= 7:
    config = {"arch": sys.argv[2], "height": int(sys.argv[3]), "width": int(sys.argv[4]),
              "frames_per_gpu_step": int(sys.argv[5]), "precision": sys.argv[6]}
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{root}/{c}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("void ", "", 1).replace("drnmi::(anonymous namespace)::", "")
            if name.endswith(")") and "(" in name:
                name = name[:name.rfind("(")]   # drop the argument list
            acc[name][c].append(float(r["Counter_Value"]))
out = {}
for k, v in acc.items():
    if not v.get("FETCH_SIZE") or not v.get("WRITE_SIZE"):
        continue
    rd = 2.0 * 1024 * sum(v["FETCH_SIZE"]) / len(v["FETCH_SIZE"])
    wr = 1024.0 * sum(v["WRITE_SIZE"]) / len(v["WRITE_SIZE"])
    out[k] = {"read_bytes": rd, "write_bytes": wr, "traffic_bytes": rd + wr, "launches": len(v["FETCH_SIZE"])}
kernels = dict(sorted(out.items(), key=lambda kv: -kv[1]["traffic_bytes"] * kv[1]["launches"]))
if config is None:
    json.dump(kernels, sys.stdout, indent=1)
else:
    json.dump({"config": config,
               "command": sys.argv[7] if len(sys.argv) > 7 else "scripts/pmc_traffic.sh",
               "correction": "read = 2 x FETCH_SIZE (gfx950 reports half of wide coalesced reads), write = "
                             "WRITE_SIZE; KB = 1024 B; per launch = mean over the kernel's dispatches; "
                             "Infinity-Cache hits included (L2<->fabric bytes)",
               "kernels": kernels}, sys.stdout, indent=1)
