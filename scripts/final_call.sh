set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash scripts/profile_round.sh ${1:-final} || exit 1
O=$R/gpurun_out/${1:-final}
timeout -k 10 200 python -u -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench failed; exit 1; }
echo all done
