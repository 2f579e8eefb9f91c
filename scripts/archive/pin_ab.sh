#!/bin/bash
# Late weight pinning A/B (GPU box): s2row / s1x2 / block64 parity tests, s2row stamps (libdrnmi_s2stamp),
# interleaved bench lines of libdrnmi (late pins) and libdrnmi_pin0 (pins before the first ring fill)
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/pin_ab; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_s2row.py tests/test_block64.py tests/test_gpu_kernels.py -k "s2row or s1x2 or fused_downsample or block64" > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
DRNMI_LIB=$R/video-seg-model-compress_amd/drnmi/libdrnmi_s2stamp.so timeout -k 10 200 python -u scripts/s2row_stamps.py 8 2>&1 | grep -v amdgpu.ids > $OUT/stamps_late.txt || exit 1
for rep in 1 2; do for lib in libdrnmi libdrnmi_pin0; do
  DRNMI_LIB=$R/video-seg-model-compress_amd/drnmi/$lib.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-exact-mode > $OUT/b_${lib}_$rep.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/b_${lib}_$rep.json').read().strip().splitlines()[-1])
ks=' '.join('%s:%.1f' % (k, v['avg_us']) for k, v in d['kernels'].items() if 's2row' in k or 's1x2' in k or 'block64' in k)
print('$lib', round(d['value'],1), round(d['ms_per_step'],3), round(d['network_roofline']['frac'],4), ks)" >> $OUT/ab.txt
done; done
cat $OUT/ab.txt; grep "per WG" $OUT/stamps_late.txt
