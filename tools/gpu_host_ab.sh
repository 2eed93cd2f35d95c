#!/bin/bash
# Host-memory build A/B (ab/libs3imph_{old,new}.so alternating): tools/host_phase.py wall
# times on C2, plus the whole -m gpu suite on the new library.   bash tools/gpu_host_ab.sh TAG
set -e
OUT=gpurun_out/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=s3-inv-db_amd/s3imph/_lib/libs3imph.so
for v in old new old new; do
  cp ab/libs3imph_$v.so $L
  timeout -k 10 200 python tools/host_phase.py >> $OUT/host_$v.log 2>&1
done
cp ab/libs3imph_new.so $L
# the new library under each A/B knob setting (AB_ENV="S3IMPH_HOST_OVERLAP=0")
for kv in $AB_ENV; do
  env $kv timeout -k 10 200 python tools/host_phase.py >> $OUT/host_knob_$kv.log 2>&1
done
timeout -k 10 200 python tools/host_phase.py 10000000 32 --debug > $OUT/host_new_debug.log 2>&1
[ -n "$NO_PYTEST" ] && { echo done > $OUT/DONE; exit 0; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1
echo done > $OUT/DONE
