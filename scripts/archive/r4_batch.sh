#!/bin/bash
# int8 on the staggered tile + fp32x fine-tune (C4) + per-kernel PMC of the bf16 step
set -u
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
O=gpurun_out/r4_batch; mkdir -p $O
bash scripts/r4_i8.sh || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -k "c4" -x -v -s --timeout 240 --timeout-method thread > $O/pytest_c4.log 2>&1 || { tail -30 $O/pytest_c4.log; exit 1; }
grep -E "C4 D-54|passed|failed" $O/pytest_c4.log | tail -4
for pr in fp32 fp32x; do
  timeout -k 10 300 python -u bench_finetune.py --precision $pr --no-cpu-baseline > $O/finetune_$pr.json 2>$O/finetune_$pr.err || { tail -5 $O/finetune_$pr.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/finetune_$pr.json').read().strip().splitlines()[-1]);print('finetune $pr', round(d['value'],2), 'img/s', round(d['ms_per_step'],1), 'ms', d['roofline']['achieved'], d['roofline']['frac'])"
done
bash scripts/pmc_bench.sh r4_batch/pmc_sq "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS" > $O/pmc_sq.txt 2>&1 || { tail -5 $O/pmc_sq.txt; exit 1; }
cat $O/pmc_sq.txt
