#!/bin/bash
# int8 layer4 (conv_w1h_i8_kernel on D-22 layer4.1 in int8 nets) bring-up: parity, then a same-box
# ABBA A/B of the int8 bench line against INT8_LAYER4 = False with diag/libdrnmi_base.so.
# usage: bash scripts/w1h_i8_ab.sh OUT
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_int8.py $R/tests/test_gpu_head_nhwc.py $R/tests/test_gpu_configs.py \
  -x -v --timeout 120 --timeout-method thread -k "int8 or i8 or c5" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
ARGS="--precision int8 --steps 40 --no-cpu-baseline"
run() {  # tag layer4
  if [ "$2" = "new" ]; then timeout -k 10 150 python3 bench.py $ARGS > $O/$1.json 2>/dev/null
  else DRNMI_LIB=$R/diag/libdrnmi_base.so timeout -k 10 150 python3 -c "
import sys, runpy
sys.path.insert(0, '$R/video-seg-model-compress_amd')
import drnmi.engine as e
e.INT8_LAYER4 = False
sys.argv = ['bench.py'] + '$ARGS'.split()
runpy.run_path('$R/bench.py', run_name='__main__')" > $O/$1.json 2>/dev/null; fi
}
for i in 1 2; do
  run new_a$i new || exit 1; run base_a$i base || exit 1
  run base_b$i base || exit 1; run new_b$i new || exit 1
done
python3 - $O <<'PY'
import json, sys, glob
rows = {}
tags = ("new", "base")
for tag in tags:
    for f in sorted(glob.glob(f"{sys.argv[1]}/{tag}_*.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        rows.setdefault(tag, []).append({l["node"]: l["us"] for l in d["layers"]})
        print(tag, round(d["value"], 1), "ms", round(d["ms_per_step"], 3), d["roofline"]["kernel"], d["roofline"]["frac"],
              "net", d.get("network_roofline", {}).get("frac"), "parity", d.get("parity_vs_ref", {}).get("label_mismatch_frac"))
keys = set(rows["base"][0]) | set(rows["new"][0])
for k in sorted(keys):
    v = [min(r.get(k, 0) for r in rows[t]) for t in tags]
    if max(v) - min(v) > 1: print(f"  {k:24s} " + "  ".join(f"{t} {x:8.1f}" for t, x in zip(tags, v)))
PY
