#!/bin/bash
# Staggered strip kernel: bit-identity tests, micro A/B (tile 18 vs 19), bench A/B (DRNMI_STAG).
set -u
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4_stag; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "stag or strip" -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
TILES=18,19 ONLY=l timeout -k 10 300 python -u scripts/conv_micro.py 8 > $O/micro.txt 2>&1 || { tail -20 $O/micro.txt; exit 1; }
cat $O/micro.txt
for rep in 1 2; do for st in 0 1; do
  DRNMI_STAG=$st timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact-mode > $O/bench_stag$st.$rep.json 2>$O/bench_stag$st.$rep.err || { tail -5 $O/bench_stag$st.$rep.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_stag$st.$rep.json').read().strip().splitlines()[-1]);print('stag$st', round(d['value'],1), d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['network_roofline']['frac'])"
done; done
