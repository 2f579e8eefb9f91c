#!/bin/bash
# Same-box A/B of bench lines across library builds, rotated order (diag/*.so are git-ignored
# builds of alternative routings; "main" = the shipped library).
# usage: bash scripts/lib_ab.sh OUT "BENCH ARGS" main libA.so libB.so ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
ARGS=$2; shift 2
LIBS=("$@")
N=${#LIBS[@]}
for rep in 0 1 2; do
  for k in $(seq 0 $((N - 1))); do
    L=${LIBS[$(( (k + rep) % N ))]}
    tag=${L%.so}
    if [ "$L" = "main" ]; then timeout -k 10 150 python3 bench.py $ARGS > $O/${tag}_$rep.json 2>/dev/null || exit 1
    else DRNMI_LIB=$R/diag/$L timeout -k 10 150 python3 bench.py $ARGS > $O/${tag}_$rep.json 2>/dev/null || exit 1; fi
  done
done
python3 - $O "${LIBS[@]}" <<'PY'
import json, sys, glob
O, libs = sys.argv[1], [l[:-3] if l.endswith(".so") else l for l in sys.argv[2:]]
rows = {}
for tag in libs:
    for f in sorted(glob.glob(f"{O}/{tag}_*.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        rows.setdefault(tag, []).append({l["node"]: l["us"] for l in d["layers"]})
        print(f"{tag:20s}", round(d["value"], 1), "ms", round(d["ms_per_step"], 3), d["roofline"]["kernel"], d["roofline"]["frac"],
              "net", round(d.get("network_roofline", {}).get("frac", 0), 4))
keys = sorted(set().union(*[set(r[0]) for r in rows.values()]))
for k in keys:
    v = [min(r.get(k, 0) for r in rows[t]) for t in libs]
    if max(v) - min(v) > 2: print(f"  {k:24s} " + "  ".join(f"{t[:10]} {x:8.1f}" for t, x in zip(libs, v)))
PY
