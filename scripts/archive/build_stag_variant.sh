#!/bin/bash
# Diagnostic-only: build drnmi/libdrnmi_<tag>.so with conv_stag.hip compiled under extra -D flags.
# usage: scripts/build_stag_variant.sh TAG -DFOO=1 ...   (select at run time with DRNMI_LIB=<path>)
set -e
tag=$1; shift
cd "$(dirname "$0")/../video-seg-model-compress_amd"
python -c "import drnmi.build as b; b.build(verbose=False)"
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I ../include "$@" -c csrc/conv_stag.hip -o build/conv_stag_$tag.o
others=$(ls build/*.hip.o | grep -v conv_stag)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/conv_stag_$tag.o $others -o drnmi/libdrnmi_$tag.so
