#!/bin/bash
set -e
OUT=gpurun_out/r3_dbg; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for kv in X=1 S3IMPH_SCAT_CFG=0 S3IMPH_MID_FENCE=1; do
  env $kv timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -q --timeout 200 --timeout-method thread -k "test_dist_host_comm_matches_oracle and 300000 and route" > $OUT/pytest_$kv.log 2>&1 || true
done
cp ab/libs3imph_old.so s3-inv-db_amd/s3imph/_lib/libs3imph.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -q --timeout 200 --timeout-method thread -k "test_dist_host_comm_matches_oracle and 300000 and route" > $OUT/pytest_old.log 2>&1 || true
echo done > $OUT/DONE
