#!/bin/bash
# A -m gpu subset, then bench lines of one config with an env knob at each value, alternating:
#   bash tools/gpu_knob_ab.sh TAG "pytest -k expr" VAR "v1 v2" [configs]   (empty -k: no tests)
set -e
OUT=gpurun_out/$1; K=$2; VAR=$3; VALS=$4; CFGS=${5:-c3}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" \
    > $OUT/pytest.log 2>&1
fi
for rep in 1 2; do
  for cfg in $CFGS; do
    for v in $VALS; do
      env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config $cfg \
        --steps 20 >> $OUT/${cfg}_$v.log 2>&1
    done
  done
done
python3 - > $OUT/summary.txt <<PY
import json, glob
for f in sorted(glob.glob("$OUT/c*_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d.get("stages_ms"))
PY
echo done > $OUT/DONE
