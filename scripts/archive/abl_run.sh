cd $GRAFT_REPO_ROOT
for lib in libdrnmi libdrnmi_abl1 libdrnmi_abl2 libdrnmi_abl3; do
  echo "== $lib"
  DRNMI_LIB=$PWD/video-seg-model-compress_amd/drnmi/$lib.so TILES=5,4 ONLY=l8 timeout -k 5 120 python scripts/conv_micro.py 8 || exit 1
  DRNMI_LIB=$PWD/video-seg-model-compress_amd/drnmi/$lib.so TILES=5,4 ONLY="l6 512x512 d4 +" timeout -k 5 120 python scripts/conv_micro.py 8 || exit 1
done
