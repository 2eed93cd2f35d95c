#!/bin/bash
# Round-end pass on one box: the whole -m gpu suite, the default bench line (C3 headline,
# C2 secondary, CPU baseline), a C5 line, and a rocprofv3 kernel-trace --stats run of the
# C3 bench command (its per-kernel averages back the bench's roofline numbers).
#   bash tools/gpu_final.sh TAG
set -e
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --durations=15 --timeout 400 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
timeout -k 10 500 python bench.py > $OUT/bench.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --headline-only --config c5 --steps 10 --warmup 2 \
  > $OUT/bench_c5.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-secondary --headline-only \
  > $OUT/bench_prof.log 2>&1
python3 tools/trace_summary.py $OUT/prof/run_kernel_trace.csv 0 > $OUT/timeline_c3.txt
echo done > $OUT/DONE
