#!/bin/bash
# GPU: default bench, then print its per-kernel breakdown (ms per step).
timeout -k 10 300 python bench.py "$@" > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
python - <<'PY'
import json
for line in open('gpurun_out/bench.log'):
    if line.startswith('{'):
        d = json.loads(line)
        print(round(d['value'], 1), 'fps', round(d['ms_per_step'], 3), 'ms/step', 'dominant', d['roofline']['kernel'],
              d['roofline']['achieved'], 'TF')
        for k, v in sorted(d['kernels'].items(), key=lambda kv: -kv[1]['launches'] * kv[1]['avg_us']):
            print(f"{k:60s} {v['launches']:4d} {v['avg_us']:8.1f} us {v['launches'] * v['avg_us'] / d['steps'] / 1000:6.3f} ms/step")
PY
