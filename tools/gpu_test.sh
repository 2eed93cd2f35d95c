#!/bin/bash
# GPU-box pass: parity tests (optionally a subset), then a short bench line.
#   bash tools/gpu_test.sh TAG [pytest -k expression]
set -e
TAG=${1:-t}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $OUT/pytest_gpu.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1
echo done > $OUT/DONE
