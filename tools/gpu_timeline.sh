#!/bin/bash
# kernel timeline of one build per config:  bash tools/gpu_timeline.sh TAG CFG [CFG...]
OUT=gpurun_out/$1; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
for cfg in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$cfg -o run -- \
    python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --headline-only $BENCH_EXTRA > $OUT/prof_$cfg.log 2>&1; rc=$?; stop $rc
  python3 tools/trace_summary.py $OUT/prof_$cfg/run_kernel_trace.csv 0 > $OUT/timeline_$cfg.txt
done
echo done >> $OUT/status
