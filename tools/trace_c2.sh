#!/bin/bash
# Kernel timeline of one C2 build (rocprofv3 kernel trace of a short bench run) plus the
# host-path tests.  bash tools/trace_c2.sh TAG [config]
set -e
OUT=gpurun_out/$1
CFG=${2:-c2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "build_host or builder" > $OUT/pytest.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/bench_prof.log 2>&1
python3 tools/trace_summary.py $OUT/prof/run_kernel_trace.csv 0 > $OUT/timeline.txt
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench.log 2>&1
echo done > $OUT/DONE
