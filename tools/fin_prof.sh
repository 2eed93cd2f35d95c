#!/bin/bash
# rocprofv3 kernel stats of the finalize pass alone (tools/fin_probe.py).  bash tools/fin_prof.sh TAG [config]
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fin -o run -- python3 tools/fin_probe.py ${2:-c3} 3 > $OUT/fin.log 2>&1
python3 - > $OUT/fin_summary.txt <<PY
import csv
for r in csv.DictReader(open("$OUT/fin/run_kernel_stats.csv")):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1][:60]
    print(f"{n:60s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:9.1f}")
PY
