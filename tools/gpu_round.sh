#!/bin/bash
# One GPU-box pass: parity tests, the default bench line, a rocprofv3 kernel-trace
# summary of the same bench command, and the two HBM PMC passes (FETCH_SIZE,
# WRITE_SIZE, each in its own run).  Usage (from the repo root, via gpurun):
#   bash tools/gpu_round.sh TAG [pytest|nopytest] [config]
set -e
TAG=${1:-run}
PYT=${2:-pytest}
CFG=${3:-c3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$PYT" = pytest ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
fi
timeout -k 10 400 python bench.py --config $CFG > $OUT/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-secondary --headline-only > $OUT/bench_prof.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --headline-only > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --headline-only > $OUT/pmc_write.log 2>&1
echo done > $OUT/DONE
