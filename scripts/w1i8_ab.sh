#!/bin/bash
# int8 conv_w1 (conv_w1_i8_kernel / conv_w1_i8_seg_kernel) bring-up: parity (oracle bits, w1 vs
# stag partials), then a same-box ABBA A/B of the int8 bench line against diag/libdrnmi_base.so
# (int8 on the staggered tile only).  usage: bash scripts/w1i8_ab.sh OUT
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_int8.py $R/tests/test_gpu_head_nhwc.py -x -v --timeout 120 \
  --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
run() {  # tag lib
  if [ "$2" = "-" ]; then timeout -k 10 150 python3 bench.py --precision int8 --steps 40 --no-cpu-baseline > $O/$1.json 2>/dev/null
  else DRNMI_LIB=$R/diag/$2 timeout -k 10 150 python3 bench.py --precision int8 --steps 40 --no-cpu-baseline > $O/$1.json 2>/dev/null; fi
}
for i in 1 2; do
  run w1_a$i - || exit 1; run base_a$i libdrnmi_base.so || exit 1
  run base_b$i libdrnmi_base.so || exit 1; run w1_b$i - || exit 1
done
python3 - $O <<'PY'
import json, sys, glob
rows = {}
tags = ("w1", "base")
for tag in tags:
    for f in sorted(glob.glob(f"{sys.argv[1]}/{tag}_*.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        rows.setdefault(tag, []).append({l["node"]: l["us"] for l in d["layers"]})
        print(tag, round(d["value"], 1), "ms", round(d["ms_per_step"], 3), d["roofline"]["kernel"], d["roofline"]["frac"],
              "net", d.get("network_roofline", {}).get("frac"))
for k in rows["base"][0]:
    v = [min(r[k] for r in rows[t]) for t in tags]
    if max(v) - min(v) > 1: print(f"  {k:24s} " + "  ".join(f"{t} {x:8.1f}" for t, x in zip(tags, v)))
PY
