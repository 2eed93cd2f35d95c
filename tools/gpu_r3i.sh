#!/bin/bash
# single-GPU C3/C2 kernel traces + the N=2 host-transport bench (alt decomposition line)
set -e
TAG=${1:-r3_i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c3 c2; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o run -- \
  python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --headline-only > $OUT/bench_$c.log 2>&1
done
bash tools/gpu_bench_multi_host.sh $TAG
