#!/bin/bash
# Per-wave phase clock of the level-0 hash (S3IMPH_DEBUG on; tools/hash_only.py), and the
# isolated kernel time under rocprofv3.  bash tools/hash_phase.sh TAG [configs]
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in ${2:-c3 c2}; do
  S3IMPH_DEBUG=1 timeout -k 10 120 python3 tools/hash_only.py $cfg 2 > $OUT/phase_$cfg.log 2>&1
  echo "$cfg $(grep -h 'hash0 wave' $OUT/phase_$cfg.log)" >> $OUT/phase_summary.txt
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$cfg -o run -- python3 tools/hash_only.py $cfg 5 > $OUT/$cfg.log 2>&1
  python3 - >> $OUT/summary.txt <<PY
import csv
rows=[r for r in csv.DictReader(open("$OUT/$cfg/run_kernel_stats.csv")) if "hash" in r["Name"]]
print("$cfg", [(r["Name"].split("(")[0].split("::")[-1][:40], round(float(r["AverageNs"])/1e3,1), r["Calls"]) for r in rows])
PY
done
