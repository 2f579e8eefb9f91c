R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r6_b64mt; mkdir -p $OUT
bash $R/scripts/gpu_tests.sh r6_b64mt tests/test_block64.py > /dev/null || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for rep in 1 2; do for lib in libdrnmi libdrnmi_b64v4; do
  echo "== $lib" >> $OUT/ab.txt
  DRNMI_LIB=$R/video-seg-model-compress_amd/drnmi/$lib.so timeout -k 5 200 python $R/scripts/block64_micro.py 2>&1 | grep -v amdgpu.ids >> $OUT/ab.txt || exit 1
done; done
cat $OUT/ab.txt
