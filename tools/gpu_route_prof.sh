#!/bin/bash
# kernel trace of the sharded (routed) build at N = 1, C3 and C2
set -e
TAG=${1:-route_prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c3 c2; do
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof_route_$c -o run -- \
  python3 bench.py --config $c --dist --decomp route --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --headline-only > $OUT/bench_route_$c.log 2>&1
done
echo done > $OUT/DONE
