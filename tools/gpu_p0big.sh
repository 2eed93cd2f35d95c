#!/bin/bash
# 64 super-tiles on 1024-thread 6144-record scatter blocks (S3IMPH_P0_BIG=1 S3IMPH_P0_MAXS=64) vs default
OUT=gpurun_out/${1:-r4_p0big}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
echo skip > $OUT/pytest.log; rc=0
echo "pytest skipped" >> $OUT/status
for rep in 1 2 3 4 5; do for v in big def; do
  if [ $v = big ]; then E="S3IMPH_P0_BIG=1 S3IMPH_P0_MAXS=64"; else E=""; fi
  env $E timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c3 --steps 20 >> $OUT/c3_$v.log 2>&1; rc=$?; stop $rc
done; done
python3 - > $OUT/summary.txt <<PY
import json, glob
for f in sorted(glob.glob("$OUT/c3_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d.get("stages_ms"))
PY
