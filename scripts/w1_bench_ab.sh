#!/bin/bash
# Same-box A/B of the bf16 bench line: the shipped library (conv_w1 routed) vs a diagnostic build
# with the staggered tile routed (diag/libdrnmi_stag.so), interleaved.  usage: bash scripts/w1_bench_ab.sh OUT
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --steps 40 --no-cpu-baseline --no-exact-mode > $O/w1_$i.json 2>/dev/null || exit 1
  DRNMI_LIB=$R/diag/libdrnmi_stag.so timeout -k 10 120 python3 bench.py --steps 40 --no-cpu-baseline --no-exact-mode > $O/stag_$i.json 2>/dev/null || exit 1
done
python3 - $O <<'PY'
import json, sys, glob
for tag in ("w1", "stag"):
    for f in sorted(glob.glob(f"{sys.argv[1]}/{tag}_*.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        ls = {l["node"]: l["us"] for l in d["layers"]}
        print(tag, round(d["value"], 1), "ms", round(d["ms_per_step"], 3), d["roofline"]["kernel"], d["roofline"]["frac"],
              "l5-8:", [ls[k] for k in ("layer.5.0.conv1", "layer.5.1.conv1", "layer.5.1.conv2", "layer.6.0.conv1", "layer.6.1.conv1", "layer.6.1.conv2", "layer.7.0", "layer.8.0")])
PY
