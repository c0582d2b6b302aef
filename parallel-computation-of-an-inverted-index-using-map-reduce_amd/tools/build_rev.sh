#!/bin/bash
# build_rev.sh NAME REV — libii_NAME.so built from the library sources of git
# revision REV (csrc/ + include/), for same-box A/B runs of tools/gpu_ab.sh
# against the working tree (II_LIB_VARIANT=NAME).
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
PKGN="parallel-computation-of-an-inverted-index-using-map-reduce_amd"
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
git -C "$ROOT" archive "$2" "$PKGN/csrc" include | tar -x -C "$TMP"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I"$TMP/include" -shared \
    -o "$ROOT/$PKGN/libii_$1.so" "$TMP/$PKGN/csrc/ii_api.hip"
