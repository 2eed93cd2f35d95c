#!/bin/bash
# parity subset per hash variant, then isolated hash kernel timings (rocprof)
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
for h in $2; do
  S3IMPH_H0=$h timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "golden or sizes or ragged or long_keys or unaligned or custom or c2_10m or level0 or repeated_builds_identical or c3_100m" > $OUT/pytest_$h.log 2>&1
  echo "h0=$h $(tail -1 $OUT/pytest_$h.log)" >> $OUT/summary.txt
done
bash tools/probe_h0.sh $1 "$2" "${3:-c3 c2}"
