#!/bin/bash
set -e
TAG=${1:-r3d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ragged or c5 or skew or repeated or bitmap" > $OUT/pytest_gpu.log 2>&1
B="python bench.py --no-cpu-baseline --no-secondary --headline-only"
timeout -k 10 300 $B --config c5 --steps 10 --warmup 2 > $OUT/c5.log 2>&1
timeout -k 10 300 python tools/skew_phase.py > $OUT/skew_phase.log 2>&1
for c in c2 c3; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o run -- \
  python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --headline-only > $OUT/bench_$c.log 2>&1
done
timeout -k 10 300 $B --config c2 --dist --decomp bitmap > $OUT/dist_c2_bitmap.log 2>&1
echo done > $OUT/DONE
