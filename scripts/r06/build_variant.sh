#!/bin/bash
# Build an A/B variant of libndfl.so: scripts/r06/build_variant.sh NAME "-DFOO=1 -DBAR" -> lib/libndfl_NAME.so
# (run on the CPU host; the variants travel to the GPU box with the tree, selected by NDFL_LIB_PATH)
set -e
cd "$(dirname "$0")/../../deflate-library-java_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -w $2 -x hip -shared -o lib/libndfl_$1.so csrc/capi/ndfl_capi.cpp
echo built lib/libndfl_$1.so
