#!/bin/bash
# super-tiles x blocks per super-tile sweep on C3 (S3IMPH_P0_TPS / S3IMPH_P0_BPS), alternating
OUT=gpurun_out/${1:-r4_sweep}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
for rep in 1 2 3 4; do for v in def 763_48 382_32 509_40; do
  if [ $v = def ]; then E=""; else E="S3IMPH_P0_TPS=${v%_*} S3IMPH_P0_BPS=${v#*_}"; fi
  env $E timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c3 --steps 20 >> $OUT/c3_$v.log 2>&1; rc=$?; stop $rc
done; done
echo done >> $OUT/status
