#!/bin/bash
# C3 phase profiles (S3IMPH_DEBUG) of the P0 super-tile scatter and of the split path's scatter0
OUT=gpurun_out/r4_p0e; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
for v in 1 0; do
  S3IMPH_DEBUG=1 S3IMPH_P0=$v timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c3 --steps 2 --warmup 1 > $OUT/dbg_p0_$v.log 2>&1; rc=$?
  echo "dbg p0=$v rc $rc" >> $OUT/status; stop $rc
done
