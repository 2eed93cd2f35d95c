#!/bin/bash
# Sharded-path (--dist, N = 1) bench lines for C3 and C2 (headline only).
#   bash tools/gpu_dist_bench.sh TAG
set -e
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 200 python bench.py --dist --no-cpu-baseline --headline-only > $OUT/bench_dist_c3.log 2>&1
timeout -k 10 200 python bench.py --dist --config c2 --no-cpu-baseline --headline-only > $OUT/bench_dist_c2.log 2>&1
echo done > $OUT/DONE
