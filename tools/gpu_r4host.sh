#!/bin/bash
# host path: new parity tests, then C2 / C3 host phases with the u16 offsets vs the old form
OUT=gpurun_out/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread \
  -k "build_host or long_keys" > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc $rc" >> $OUT/status; stop $rc
for v in 1 0; do
  S3IMPH_OFF16=$v timeout -k 10 200 python tools/host_phase.py 10000000 32 > $OUT/host_c2_off16_$v.log 2>&1; rc=$?; stop $rc
  S3IMPH_OFF16=$v timeout -k 10 300 python tools/host_phase.py 100000000 64 > $OUT/host_c3_off16_$v.log 2>&1; rc=$?; stop $rc
done
S3IMPH_DEBUG=1 timeout -k 10 300 python tools/host_phase.py 100000000 64 > $OUT/host_c3_dbg.log 2>&1; rc=$?; stop $rc
grep -h "build_host" $OUT/host_c*_off16_*.log > /dev/null
for f in $OUT/host_c*_off16_*.log; do echo "$f $(grep build_host $f | tail -5 | awk '{print $3}' | tr '\n' ' ')"; done > $OUT/summary.txt
