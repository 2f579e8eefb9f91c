set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_kernels.py tests/test_gpu_int8.py tests/test_gpu_sparse.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || { tail -20 gpurun_out/ab/pytest.log; exit 1; }
tail -1 gpurun_out/ab/pytest.log
for rep in 1 2; do
for lib in libdrnmi_$1 libdrnmi; do
  DRNMI_LIB=$PWD/video-seg-model-compress_amd/drnmi/$lib.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "${@:2}" > gpurun_out/ab/$lib.$rep.json 2>/dev/null || exit 1
  python -c "import json,sys;d=json.loads(open('gpurun_out/ab/$lib.$rep.json').read().strip().splitlines()[-1]);print('$lib', round(d['value'],1), d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done; done
