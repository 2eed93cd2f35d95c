#!/bin/bash
# Round-2 hash sweep: parity subset under each candidate variant, then bench lines per variant.
set -e
OUT=gpurun_out/$1
VARS=${2:-"1 5 6"}
CFGS=${3:-"c2 c3"}
mkdir -p $OUT
for h in $VARS; do
  S3IMPH_H0=$h timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "golden or sizes or ragged or long_keys or unaligned or custom or c2_10m or level0 or repeated_builds_identical or c3_100m or duplicate" > $OUT/pytest_$h.log 2>&1
  tail -1 $OUT/pytest_$h.log >> $OUT/summary.txt
done
for cfg in $CFGS; do
  for h in $VARS; do
    S3IMPH_H0=$h timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --config $cfg --steps 10 --warmup 2 > $OUT/b_${cfg}_$h.log 2>&1
    python3 -c "import json,sys; d=json.loads(open('$OUT/b_${cfg}_$h.log').read().strip().splitlines()[-1]); print('$cfg h0=$h', round(d['ms_per_step'],3), d['stages_ms'].get('hash_count0'))" >> $OUT/summary.txt
  done
done
