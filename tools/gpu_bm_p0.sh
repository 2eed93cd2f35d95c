#!/bin/bash
# bitmap decomposition with the P0 level 0: GPU tests (multi + dist), then C3 / C2 at N = 1
OUT=gpurun_out/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_dist.py -m gpu -v --timeout 400 \
  --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc $rc" >> $OUT/status; stop $rc
BENCH_EXTRA="--dist --decomp bitmap" bash tools/gpu_ab_env.sh $1/bm c3 2 - S3IMPH_P0=0
