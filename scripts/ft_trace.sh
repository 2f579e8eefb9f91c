#!/bin/bash
# fine-tune (C4) kernel trace: the fp32x bench line and a per-dispatch rocprofv3 trace of it.
# usage: bash scripts/ft_trace.sh OUT
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python3 $R/bench_finetune.py --precision fp32x --no-cpu-baseline > $O/ft_bench.json 2> $O/ft_bench.err || { tail -5 $O/ft_bench.err; exit 1; }
tail -c 600 $O/ft_bench.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 $R/bench_finetune.py --precision fp32x --no-cpu-baseline --steps 3 --warmup 1 > $O/ft_rocprof.log 2>&1) || { echo trace failed; exit 1; }
echo done
