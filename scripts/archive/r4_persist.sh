#!/bin/bash
# persistent 128-channel stag tile: tests under both settings, bench A/B (DRNMI_STAG_PERSIST)
set -u
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4_persist; mkdir -p $O
for pv in 0 1; do
DRNMI_STAG_PERSIST=$pv timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "stag or fused_downsample" -x -q --timeout 120 --timeout-method thread > $O/pytest$pv.log 2>&1 || { tail -30 $O/pytest$pv.log; exit 1; }
echo "persist=$pv $(tail -1 $O/pytest$pv.log)"
done
for rep in 1 2; do for pv in 0 1; do
  DRNMI_STAG_PERSIST=$pv timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact-mode > $O/bench_p$pv.$rep.json 2>$O/err || { tail -5 $O/err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_p$pv.$rep.json').read().strip().splitlines()[-1]);k=d['kernels'];print('persist$pv', round(d['value'],1), round(d['network_roofline']['frac'],4), [(n[:24],v['launches'],v['avg_us']) for n,v in k.items() if '128' in n])"
done; done
