#!/bin/bash
# A/B of an environment knob: parity subset + bench stages per value.
#   bash tools/ab_env.sh TAG VAR "v1 v2" [config] [pytest -k expr]
set -e
OUT=gpurun_out/$1
VAR=$2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in $3; do
  if [ -n "$5" ]; then
    env $VAR=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
      -k "$5" > $OUT/pytest_$v.log 2>&1
    echo "$VAR=$v $(tail -1 $OUT/pytest_$v.log)" >> $OUT/summary.txt
  fi
  env $VAR=$v timeout -k 10 300 python bench.py --config ${4:-c3} --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > $OUT/b_$v.log 2>&1
  python3 - >> $OUT/summary.txt <<PY
import json
d = json.loads(open("$OUT/b_$v.log").read().strip().splitlines()[-1])
print("$VAR=$v", round(d["ms_per_step"], 3), d["stages_ms"])
PY
done
