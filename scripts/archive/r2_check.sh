#!/bin/bash
# Round-2 GPU check: full GPU suite (with prints), smoke, bf16 / fp32 / host-frames bench lines.
# usage: bash scripts/r2_check.sh OUTNAME
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $R/tests -x -v -s -m gpu --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/pytest_gpu.log; tail -4 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u $R/bench.py > $OUT/bench_bf16.json 2> $OUT/bench_bf16.err || { echo bench bf16 failed; tail -5 $OUT/bench_bf16.err; exit 1; }
timeout -k 10 300 python -u $R/bench.py --precision fp32 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_fp32.json 2> $OUT/bench_fp32.err || { echo bench fp32 failed; exit 1; }
timeout -k 10 300 python -u $R/bench.py --host-frames --no-cpu-baseline > $OUT/bench_host.json 2> $OUT/bench_host.err || { echo bench host failed; exit 1; }
python3 - <<PY
import json
for n in ("bf16", "fp32", "host"):
    d = json.loads(open("$OUT/bench_%s.json" % n).read().strip().splitlines()[-1])
    print(n, round(d["value"], 1), d["roofline"]["kernel"], d["roofline"]["frac"], d.get("host_frames", {}).get("value"),
          d.get("cpu_baseline", {}).get("value"), d.get("cpu_baseline", {}).get("cores"))
PY
