#!/bin/bash
# Same-box A/B of the bf16 bench line: the shipped library (conv_w1h routed on the short-K
# launches) vs the previous routing (diag/libdrnmi_base.so), interleaved.  usage: bash scripts/w1h_bench_ab.sh OUT
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --steps 40 --no-cpu-baseline --no-exact-mode > $O/w1h_$i.json 2>/dev/null || exit 1
  DRNMI_LIB=$R/diag/libdrnmi_base.so timeout -k 10 120 python3 bench.py --steps 40 --no-cpu-baseline --no-exact-mode > $O/base_$i.json 2>/dev/null || exit 1
done
python3 - $O <<'PY'
import json, sys, glob
rows = {}
for tag in ("w1h", "base"):
    for f in sorted(glob.glob(f"{sys.argv[1]}/{tag}_*.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        ls = {l["node"]: l["us"] for l in d["layers"]}
        rows.setdefault(tag, []).append(ls)
        print(tag, round(d["value"], 1), "ms", round(d["ms_per_step"], 3), d["roofline"]["kernel"], d["roofline"]["frac"],
              "net", d.get("network_roofline", {}).get("frac"))
for k in rows["w1h"][0]:
    a = min(r[k] for r in rows["w1h"]); b = min(r[k] for r in rows["base"])
    if abs(a - b) > 1: print(f"  {k:24s} w1h {a:8.1f}  base {b:8.1f}")
PY
