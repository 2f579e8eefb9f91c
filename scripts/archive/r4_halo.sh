#!/bin/bash
# 128-channel staggered tile vs the halo kernel for D-22 layer4: bit-identity, bench A/B (DRNMI_HALO)
set -u
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4_halo; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "stag or fused_downsample or halo or strip" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do for hv in 1 0; do
  DRNMI_HALO=$hv timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact-mode > $O/bench_halo$hv.$rep.json 2>$O/err || { tail -5 $O/err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_halo$hv.$rep.json').read().strip().splitlines()[-1]);k=d['kernels'];print('halo$hv', round(d['value'],1), round(d['network_roofline']['frac'],4), [(n[:24],v['launches'],v['avg_us']) for n,v in k.items() if 'halo' in n or '128' in n])"
done; done
