#!/bin/bash
# Diagnostic-only: build drnmi/libdrnmi_<tag>.so with one csrc source compiled under extra -D flags.
# usage: scripts/build_variant_src.sh TAG SRC.hip -DFOO=1 ...   (select at run time with DRNMI_LIB=<path>)
set -e
tag=$1; src=$2; shift 2
cd "$(dirname "$0")/../video-seg-model-compress_amd"
python -c "import drnmi.build as b; b.build(verbose=False)"
base=$(basename $src .hip)
extra=$(python -c "import drnmi.build as b; print(' '.join(b.EXTRA.get('$src', [])))")
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I ../include $extra "$@" -c csrc/$src -o build/${base}_$tag.o
others=$(ls build/*.hip.o | grep -v "/$base.hip.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/${base}_$tag.o $others -o drnmi/libdrnmi_$tag.so
