#!/bin/bash
# A/B of two library builds on one box: ab/libs3imph_{old,new}.so, alternating, with the
# given bench arguments.   bash tools/gpu_ab.sh TAG "bench args"
set -e
OUT=gpurun_out/$1; mkdir -p $OUT
L=s3-inv-db_amd/s3imph/_lib/libs3imph.so
for v in old new old new; do
  cp ab/libs3imph_$v.so $L
  timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only $2 >> $OUT/$v.log 2>&1
done
cp ab/libs3imph_new.so $L
echo done > $OUT/DONE
