#!/bin/bash
set -e
TAG=${1:-r3c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "dist or multi" > $OUT/pytest_gpu.log 2>&1
B="python bench.py --no-cpu-baseline --no-secondary --headline-only"
for d in route bitmap; do
  timeout -k 10 300 $B --config c2 --dist --decomp $d > $OUT/dist_c2_$d.log 2>&1
  timeout -k 10 300 $B --config c3 --dist --decomp $d --steps 10 --warmup 2 > $OUT/dist_c3_$d.log 2>&1
done
timeout -k 10 300 python tools/skew_phase.py > $OUT/skew_phase.log 2>&1
echo done > $OUT/DONE
