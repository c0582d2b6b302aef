#!/bin/bash
# build_variant.sh NAME "-DFLAG=1 ..." — libii_NAME.so: libii.so built with extra
# defines, for tools/gpu_ab.sh (loaded through II_LIB_VARIANT=NAME).
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
PKG="$ROOT/parallel-computation-of-an-inverted-index-using-map-reduce_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I"$ROOT/include" $2 -shared \
    -o "$PKG/libii_$1.so" "$PKG/csrc/ii_api.hip"
