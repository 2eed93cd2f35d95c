#!/bin/bash
# A/B of env settings on one config:  bash tools/gpu_ab_env.sh TAG CONFIG REPS "ENV_A" "ENV_B" ...
# (each ENV is a space-separated list of VAR=VALUE, or "-" for none); stage times -> summary.txt
OUT=gpurun_out/$1; CFG=$2; REPS=$3; shift 3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
for rep in $(seq $REPS); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    envs=""; [ "$e" != "-" ] && envs="$e"
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config $CFG --steps 20 $BENCH_EXTRA >> $OUT/v$i.log 2>&1; rc=$?
    echo "v$i ($e) rep $rep rc $rc" >> $OUT/status; stop $rc
  done
done
python3 - "$OUT" "$@" > $OUT/summary.txt <<'PY'
import json, sys
out = sys.argv[1]
for i, e in enumerate(sys.argv[2:], 1):
    for line in open(f"{out}/v{i}.log"):
        if line.startswith("{"):
            d = json.loads(line)
            print(f"v{i} [{e}]", round(d["ms_per_step"], 4), d.get("stages_ms"))
PY
