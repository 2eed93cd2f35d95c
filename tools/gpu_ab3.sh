#!/bin/bash
# Round-3 A/B pass: parity tests on the touched paths, then bench lines for C3 / C5 / C2
# and the sharded path at N = 1 with both decompositions (route, bitmap) on C2 and C3,
# and a kernel trace of the C3 headline.   bash tools/gpu_ab3.sh TAG ["pytest -k expr"]
set -e
TAG=${1:-ab}
K=${2:-"parity or scale or dist or multi"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "$K" > $OUT/pytest_gpu.log 2>&1
B="python bench.py --no-cpu-baseline --no-secondary --headline-only"
timeout -k 10 300 $B --config c3 > $OUT/c3.log 2>&1
timeout -k 10 300 $B --config c5 --steps 10 --warmup 2 > $OUT/c5.log 2>&1
timeout -k 10 300 $B --config c2 > $OUT/c2.log 2>&1
for d in route bitmap; do
  timeout -k 10 300 $B --config c2 --dist --decomp $d > $OUT/dist_c2_$d.log 2>&1
  timeout -k 10 300 $B --config c3 --dist --decomp $d --steps 10 --warmup 2 > $OUT/dist_c3_$d.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --headline-only > $OUT/prof.log 2>&1
echo done > $OUT/DONE
