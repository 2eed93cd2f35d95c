#!/bin/bash
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./tools/ubench_ops.bin > $OUT/ubench_ops.txt 2>&1
for cfg in ${3:-c3 c2}; do
  for h in ${2:-0 1 3 5 7 8}; do
    S3IMPH_H0=$h timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${cfg}_$h -o run -- python3 tools/hash_only.py $cfg 5 > $OUT/${cfg}_$h.log 2>&1
    python3 - >> $OUT/summary.txt <<PY
import csv
rows=[r for r in csv.DictReader(open("$OUT/${cfg}_$h/run_kernel_stats.csv")) if "hash" in r["Name"]]
print("$cfg h0=$h", [(r["Name"].split("(")[0].split("::")[-1][:40], round(float(r["AverageNs"])/1e3,1), r["Calls"]) for r in rows])
PY
  done
done
