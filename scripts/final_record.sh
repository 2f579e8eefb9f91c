#!/bin/bash
# Final-tree record: full GPU suite, smoke, every bench line (bf16 headline with exact_mode, fp32,
# fp32x, int8, int8 + SRMB (C5), host frames, C3 block-sparse 16x16 dense/sparse, fine-tune fp32 /
# fp32x).  usage: bash scripts/final_record.sh OUTNAME
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $R/tests -x -v -s -m gpu --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/pytest_gpu.log; tail -3 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
b() { local name=$1; shift; timeout -k 10 300 python -u $R/bench.py "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { echo "bench $name failed"; tail -5 $OUT/bench_$name.err; exit 1; }; }
b bf16
b fp32 --precision fp32 --steps 5 --warmup 2 --no-cpu-baseline
b fp32x --precision fp32x --steps 5 --warmup 2
b int8 --precision int8 --no-cpu-baseline
b int8_srmb --precision int8 --prune json:tests/golden/srmb_d22_1024X768_50.json --no-cpu-baseline
b host --host-frames --no-cpu-baseline
b c3_16x16_dense --arch drn_d_38 --prune block:16x16:0.5 --steps 10 --warmup 3 --no-cpu-baseline --no-exact-mode
b c3_16x16_sparse --arch drn_d_38 --prune block:16x16:0.5 --block-sparse --steps 10 --warmup 3 --no-cpu-baseline --no-exact-mode
timeout -k 10 300 python -u $R/bench_finetune.py --cpu-seconds 10 > $OUT/finetune_fp32.json 2> $OUT/finetune_fp32.err || { echo ft fp32 failed; exit 1; }
timeout -k 10 300 python -u $R/bench_finetune.py --precision fp32x --no-cpu-baseline > $OUT/finetune_fp32x.json 2> $OUT/finetune_fp32x.err || { echo ft fp32x failed; exit 1; }
python3 - <<PY
import glob, json, os
for f in sorted(glob.glob("$OUT/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print(os.path.basename(f), round(d["value"], 2), d["unit"], r.get("kernel"), r.get("frac"),
          d.get("network_roofline", {}).get("frac"), (d.get("parity_vs_ref") or {}).get("label_agreement"))
PY
