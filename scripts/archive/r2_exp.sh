#!/bin/bash
# Round-2 kernel experiment: selected GPU tests, a bench line, then PMC passes over a short bench.
# usage: bash scripts/r2_exp.sh OUTNAME "pytest -k expr" [pmc]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests -x -q -m gpu -k "$2" --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { tail -30 $OUT/pytest.log; exit $rc; }
timeout -k 10 200 python -u $R/bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -5 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(round(d['value'],1), d['ms_per_step'])
for k,v in list(d['kernels'].items())[:14]: print(' ', k, v)"
if [ "${3:-}" = pmc ]; then
  bash $R/scripts/pmc_cmd.sh $1/pmc bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null || exit 1
  python3 $R/scripts/pmc_table.py $OUT/pmc "${PMC_FILTER:-}" > $OUT/pmc_table.txt
fi
echo ok
