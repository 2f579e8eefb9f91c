#!/bin/bash
# int8 (C5) on the staggered tile: oracle bit-exactness, then bench A/B stag vs strip, SRMB line
set -u
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4_i8; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_int8.py tests/test_gpu_configs.py -k "i8 or c5" -x -v -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
for rep in 1 2; do for st in 0 1; do
  DRNMI_STAG=$st timeout -k 10 200 python bench.py --precision int8 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_int8_stag$st.$rep.json 2>$O/err || { tail -5 $O/err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_int8_stag$st.$rep.json').read().strip().splitlines()[-1]);print('int8 stag$st', round(d['value'],1), d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done; done
timeout -k 10 200 python bench.py --precision int8 --prune json:tests/golden/srmb_d22_1024X768_50.json --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_int8_srmb.json 2>$O/err || { tail -5 $O/err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_int8_srmb.json').read().strip().splitlines()[-1]);print('int8 srmb', round(d['value'],1), d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
