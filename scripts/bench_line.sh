#!/bin/bash
# One bench.py line with its per-kernel table: bash scripts/bench_line.sh OUTNAME TAG [bench args...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; TAG=$2; shift 2
mkdir -p $OUT
timeout -k 10 300 python -u $R/bench.py "$@" > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench $TAG failed"; tail -5 $OUT/bench_$TAG.err; exit 1; }
python3 - "$OUT/bench_$TAG.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"])
for k, v in d.get("kernels", {}).items():
    print("  ", k, v)
print(d.get("network_roofline"))
PY
