#!/bin/bash
# P0 / tile subset tests, then C3 (x2) and C2 (x2) stage times, then the level-1 ts A/B
OUT=gpurun_out/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  -k "p0 or big_tiles or c3_100m_bit_exact or c5_one_gpu_share or c4_one_gpu_share or dup or repeated or sizes or build_host" > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc $rc" >> $OUT/status; stop $rc
bash tools/gpu_ab_env.sh $1/c3 c3 2 - S3IMPH_TS_MAX=5 S3IMPH_PT_DIRECT=1 && bash tools/gpu_ab_env.sh $1/c2 c2 2 -
