#!/bin/bash
set -e
TAG=${1:-r3e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ragged or c5 or c3 or c2 or repeated or golden or sizes or dist_unbalanced" > $OUT/pytest_gpu.log 2>&1
B="python bench.py --no-cpu-baseline --no-secondary --headline-only"
timeout -k 10 300 $B --config c5 --steps 10 --warmup 2 > $OUT/c5.log 2>&1
timeout -k 10 300 $B --config c3 > $OUT/c3.log 2>&1
timeout -k 10 300 $B --config c2 > $OUT/c2.log 2>&1
timeout -k 10 300 python tools/skew_phase.py > $OUT/skew_phase.log 2>&1
echo done > $OUT/DONE
