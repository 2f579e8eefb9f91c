#!/bin/bash
# Diagnostic-only builds of libdrnmi.so with conv_big.hip compiled under DRNMI_ABLATE=N
# (bit 0: no in-loop DMA, bit 1: no MFMA).  Outputs drnmi/libdrnmi_abl{1,2,3}.so (git-ignored);
# select one at run time with DRNMI_LIB=<path>.  Never shipped.
set -e
cd "$(dirname "$0")/../video-seg-model-compress_amd"
python -c "import drnmi.build as b; b.build()"
for n in 1 2 3; do
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I ../include -DDRNMI_ABLATE=$n \
    -c csrc/conv_big.hip -o build/conv_big_abl$n.o &
done
wait
others=$(ls build/*.hip.o | grep -v conv_big)
for n in 1 2 3; do
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/conv_big_abl$n.o $others -o drnmi/libdrnmi_abl$n.so
done
