#!/bin/bash
# GPU-box pass over the other bench configurations (C3, C4, C5, the multi-GPU path
# at N=1) plus the driver's smoke(); one bench line per config under gpurun_out/TAG.
#   bash tools/gpu_configs.sh TAG
set -e
TAG=${1:-cfg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
for cfg in c3 c4 c5; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $cfg --steps 10 --warmup 2 > $OUT/bench_$cfg.log 2>&1
done
timeout -k 10 300 python bench.py --no-cpu-baseline --dist --steps 20 --warmup 3 > $OUT/bench_dist1.log 2>&1
echo done > $OUT/DONE
