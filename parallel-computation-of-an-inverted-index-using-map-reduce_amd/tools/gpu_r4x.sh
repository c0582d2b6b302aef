#!/bin/bash
# one session: the side-stream long-word check's grid (II_LV_BLOCKS 128 / 32 / 8 builds) — it overlaps the
# dictionary's slot compaction on the critical path — at config3, then the collision test with the smallest
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4x}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests (lv8)" && \
II_LIB_VARIANT=lv8 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "collision or long_word or tiny_shapes or map_host" > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
bash $T/gpu_env_ab.sh $TAG 10e9 10 - II_LIB_VARIANT=lv32 II_LIB_VARIANT=lv8 - II_LIB_VARIANT=lv32 II_LIB_VARIANT=lv8
