#!/bin/bash
# same-box A/B of the list-level geometry bounds (tight default vs S3IMPH_LOOSE_GEOM), C3 and C2,
# interleaved twice
set -e
OUT=gpurun_out/${1:-ab_geom}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --no-cpu-baseline --no-secondary --headline-only"
for i in 1 2; do
  timeout -k 10 200 $B --config c3 > $OUT/c3_tight_$i.log 2>&1
  S3IMPH_LOOSE_GEOM=1 timeout -k 10 200 $B --config c3 > $OUT/c3_loose_$i.log 2>&1
  timeout -k 10 200 $B --config c2 > $OUT/c2_tight_$i.log 2>&1
  S3IMPH_LOOSE_GEOM=1 timeout -k 10 200 $B --config c2 > $OUT/c2_loose_$i.log 2>&1
done
echo done > $OUT/DONE
