#!/bin/bash
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
for cfg in c3 c2; do
  S3IMPH_DEBUG=1 S3IMPH_H0=1 timeout -k 10 120 python3 tools/hash_only.py $cfg 2 > $OUT/$cfg.log 2>&1
done
grep -h "hash0 waves" $OUT/*.log > $OUT/summary.txt || true
