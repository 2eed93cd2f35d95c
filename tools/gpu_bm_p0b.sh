#!/bin/bash
OUT=gpurun_out/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
S3IMPH_DEBUG=1 S3IMPH_DIST_STRICT=1 timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c3 --steps 2 --warmup 1 --dist --decomp bitmap > $OUT/dbg_c3.log 2>&1; rc=$?; echo "dbg rc $rc" >> $OUT/status; stop $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_dist.py -m gpu -v --timeout 400 \
  --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc $rc" >> $OUT/status; stop $rc
