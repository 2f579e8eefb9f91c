#!/bin/bash
# Stag variants: bit-identity per library, then interleaved micro A/B on the layer5-8 shapes (tile 19)
set -u
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4_stagvar; mkdir -p $O
D=$PWD/video-seg-model-compress_amd/drnmi
for lib in libdrnmi "$@"; do
  DRNMI_LIB=$D/$lib.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "stag or fused_downsample" -x -q --timeout 120 --timeout-method thread > $O/pytest_$lib.log 2>&1 || { echo "FAIL $lib"; tail -30 $O/pytest_$lib.log; exit 1; }
  echo "$lib: $(tail -1 $O/pytest_$lib.log)"
done
for rep in 1 2; do for lib in libdrnmi "$@"; do
  echo "== $lib"
  DRNMI_LIB=$D/$lib.so TILES=19 ONLY=l timeout -k 10 200 python scripts/conv_micro.py 8 2>/dev/null | head -5 || exit 1
done; done
for rep in 1 2; do for lib in libdrnmi "$@"; do
  DRNMI_LIB=$D/$lib.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact-mode > $O/bench_$lib.$rep.json 2>$O/bench_$lib.$rep.err || { tail -5 $O/bench_$lib.$rep.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$lib.$rep.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$lib', round(d['value'],1), d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'], round(d['network_roofline']['frac'],4), [(n[:20],v['avg_us']) for n,v in k.items() if 'x2' in n or 'true>' in n])"
done; done
