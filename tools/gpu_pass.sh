#!/bin/bash
# One GPU-box pass: the whole -m gpu suite (per-test timeout), then the default bench line
# (C3 headline + C2 secondary with the host / builder end-to-end numbers) and a C5 line.
#   bash tools/gpu_pass.sh TAG [pytest -k expression]
set -e
TAG=${1:-pass}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$K" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "$K" > $OUT/pytest_gpu.log 2>&1
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
fi
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --headline-only --config c5 --steps 10 --warmup 2 > $OUT/bench_c5.log 2>&1
echo done > $OUT/DONE
