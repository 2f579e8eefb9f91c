#!/bin/bash
# conv_x6 change bring-up: fp32x / fine-tune parity, the x6 micro (SHA of every output: bit
# identity), then rotated-order A/B of the fp32x bench line and the fine-tune line against
# diag/libdrnmi_base.so.  usage: bash scripts/x6_ab.sh OUT
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 500 python -u -m pytest $R/tests/test_gpu_kernels.py $R/tests/test_gpu_forward.py $R/tests/test_gpu_train.py \
  $R/tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -k "x6 or fp32x or c1 or c4 or train" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 $R/scripts/x6_micro.py > $O/micro_new.log 2>&1 || exit 1
DRNMI_LIB=$R/diag/libdrnmi_base.so timeout -k 10 120 python3 $R/scripts/x6_micro.py > $O/micro_base.log 2>&1 || exit 1
for rep in 0 1; do
  timeout -k 10 200 python3 bench.py --precision fp32x --steps 10 --warmup 3 --no-cpu-baseline > $O/x_new_$rep.json 2>/dev/null || exit 1
  DRNMI_LIB=$R/diag/libdrnmi_base.so timeout -k 10 200 python3 bench.py --precision fp32x --steps 10 --warmup 3 --no-cpu-baseline > $O/x_base_$rep.json 2>/dev/null || exit 1
  DRNMI_LIB=$R/diag/libdrnmi_base.so timeout -k 10 200 python3 bench_finetune.py --precision fp32x --no-cpu-baseline > $O/ft_base_$rep.json 2>/dev/null || exit 1
  timeout -k 10 200 python3 bench_finetune.py --precision fp32x --no-cpu-baseline > $O/ft_new_$rep.json 2>/dev/null || exit 1
done
python3 - $O <<'PY'
import json, sys, glob
O = sys.argv[1]
for pat in ("x_new", "x_base", "ft_new", "ft_base"):
    for f in sorted(glob.glob(f"{O}/{pat}_*.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(pat, round(d["value"], 2), round(d["ms_per_step"], 3), d["roofline"].get("kernel", "")[:40], d["roofline"]["frac"])
new = [l.split() for l in open(f"{O}/micro_new.log") if "sha" in l]
old = [l.split() for l in open(f"{O}/micro_base.log") if "sha" in l]
for a, b in zip(new, old):
    ua, ub = [t for t in a if t.endswith("us")], [t for t in b if t.endswith("us")]
    print(" ".join(a[:4])[:50], "new", a[a.index("us") - 1] if "us" in a else ua, "base", b[b.index("us") - 1] if "us" in b else ub,
          "same" if a[-1] == b[-1] else "DIFF")
PY
