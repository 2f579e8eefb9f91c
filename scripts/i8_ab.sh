#!/bin/bash
# int8 bench A/B over tile-variant overrides, interleaved on one box, with the per-kernel times:
#   bash scripts/i8_ab.sh OUT "V1=-1,V3=-1 V1=0,V3=-1 ..." [bench args]
# (DRNMI_I8_V1 / DRNMI_I8_V3: csrc/conv_big.hip i8_variant; -1 = the default pick)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; CFGS=$2; shift 2
mkdir -p $OUT
for rep in 1 2; do
for c in $CFGS; do
  v1=$(echo $c | sed 's/.*V1=\([-0-9]*\).*/\1/'); v3=$(echo $c | sed 's/.*V3=\([-0-9]*\).*/\1/')
  DRNMI_I8_V1=$v1 DRNMI_I8_V3=$v3 timeout -k 10 200 python -u $R/bench.py --precision int8 --no-cpu-baseline \
      --no-exact-mode "$@" > $OUT/b_${c}_$rep.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/b_${c}_$rep.json').read().strip().splitlines()[-1])
ks=' '.join('%s:%.1fx%d' % (k.replace('conv_i8_kernel', 'i8'), v['avg_us'], v['launches']) for k, v in d['kernels'].items() if 'i8' in k or 'halo' in k or 'block64' in k)
print('$c', round(d['value'],1), round(d['ms_per_step'],3), d['network_roofline']['frac'], ks)" >> $OUT/ab.txt
done; done
cat $OUT/ab.txt
