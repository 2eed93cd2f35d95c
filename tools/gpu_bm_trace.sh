#!/bin/bash
# bitmap decomposition at N=1 on C3: bench line + one kernel timeline (gaps = host round trips)
OUT=gpurun_out/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "bitmap or build_host or dist" > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc $rc" >> $OUT/status; stop $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c3 --steps 10 --dist --decomp bitmap > $OUT/bm_c3.log 2>&1; rc=$?; stop $rc
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/prof_bm -o run -- \
  python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --headline-only --dist --decomp bitmap > $OUT/prof_bm.log 2>&1; rc=$?; stop $rc
python3 tools/trace_summary.py $OUT/prof_bm/run_kernel_trace.csv 0 > $OUT/timeline_bm.txt
echo done >> $OUT/status
