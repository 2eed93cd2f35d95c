#!/bin/bash
OUT=gpurun_out/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_dist.py tests/test_gpu_parity.py -m gpu -v --timeout 400 \
  --timeout-method thread -k "p0 or bitmap or dist or thread or rccl or builder" > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc $rc" >> $OUT/status; stop $rc
BENCH_EXTRA="--dist --decomp bitmap" bash tools/gpu_ab_env.sh $1/bm c3 2 -
bash tools/gpu_ab_env.sh $1/c3 c3 1 -
