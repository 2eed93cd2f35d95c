#!/bin/bash
set -e
TAG=${1:-bmprof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "bitmap or dist or multi" > $OUT/pytest_gpu.log 2>&1
for c in c2 c3; do
S3IMPH_DIST_STRICT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o run -- \
  python3 bench.py --config $c --dist --decomp bitmap --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --headline-only > $OUT/bench_$c.log 2>&1
timeout -k 10 300 python3 bench.py --config $c --dist --decomp route --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --headline-only > $OUT/bench_route_$c.log 2>&1
done
echo done > $OUT/DONE
