#!/bin/bash
# Kernel timelines (rocprofv3 kernel trace) of one C3 and one C2 build, plus the debug
# phase profiles (S3IMPH_DEBUG) of both.   bash tools/gpu_timeline.sh TAG
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in c3 c2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$cfg -o run -- \
    python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --headline-only \
    > $OUT/bench_prof_$cfg.log 2>&1
  python3 tools/trace_summary.py $OUT/prof_$cfg/run_kernel_trace.csv 0 > $OUT/timeline_$cfg.txt
done
timeout -k 10 200 python3 tools/c3_debug.py > $OUT/debug_c3.log 2>&1
timeout -k 10 200 python3 tools/c3_debug.py 10000000 32 > $OUT/debug_c2.log 2>&1
echo done > $OUT/DONE
