#!/bin/bash
# Round-end pass on one box (tools/gpu.sh steps): the whole -m gpu suite, the default bench
# line (C3 headline, C2 secondary, CPU baseline), a C5 line, the bitmap decomposition at N = 1,
# and a rocprofv3 kernel-trace --stats run of the C3 bench command (its per-kernel averages back
# the bench's roofline numbers).
#   bash tools/gpu_final.sh TAG
T=${1:-final}
bash tools/gpu.sh $T pytest &&
bash tools/gpu.sh $T bench bench &&
bash tools/gpu.sh $T bench bench_c5 --no-cpu-baseline --no-secondary --headline-only --config c5 --steps 10 --warmup 2 &&
bash tools/gpu.sh $T bench bench_bm1 --no-cpu-baseline --no-secondary --headline-only --dist --decomp bitmap --steps 10 &&
bash tools/gpu.sh $T prof c3 --config c3
