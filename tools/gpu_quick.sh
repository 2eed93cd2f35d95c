#!/bin/bash
# Short GPU-box pass: selected test files, then the default bench line (no CPU baseline).
#   bash tools/gpu_quick.sh TAG "tests/test_a.py tests/test_b.py" [bench args]
set -e
TAG=${1:-q}
FILES=${2:-tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest $FILES -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline ${3:-} > $OUT/bench.log 2>&1
echo done > $OUT/DONE
