#!/bin/bash
# Full GPU test suite on the in-tree build, then an A/B of ab/libs3imph_{old,new}.so.
#   bash tools/gpu_test_ab.sh TAG "bench args"
set -e
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
bash tools/gpu_ab.sh $1ab "$2"
