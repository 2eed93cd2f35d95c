#!/bin/bash
# super-tile count / blocks per super-tile: default (64 x 8) vs 48 x 16 (S3IMPH_P0_TPS=256 S3IMPH_P0_BPS=16)
OUT=gpurun_out/${1:-r4_s48}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
S3IMPH_P0_TPS=256 S3IMPH_P0_BPS=16 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "c3_100m" > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc $rc" >> $OUT/status; stop $rc; [ $rc = 0 ] || exit $rc
for rep in 1 2 3 4; do for v in s48 def; do
  if [ $v = s48 ]; then E="S3IMPH_P0_TPS=256 S3IMPH_P0_BPS=16"; else E=""; fi
  env $E timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c3 --steps 20 >> $OUT/c3_$v.log 2>&1; rc=$?; stop $rc
done; done
