#!/bin/bash
# Full -m gpu suite on the in-tree build, then an old/new library A/B (abx/libs3imph_{old,new}.so,
# alternating) on C2 and C3.   bash tools/gpu_ab_full.sh TAG [pytest -k expr]
set -e
OUT=gpurun_out/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$2" > $OUT/pytest.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
fi
# correctness of an A/B knob (PYT_ENV="S3IMPH_MID_HS=1"): the parity and dist files under it
if [ -n "$PYT_ENV" ]; then
  env $PYT_ENV timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest_knob.log 2>&1 || true
fi
L=s3-inv-db_amd/s3imph/_lib/libs3imph.so
for cfg in ${CFGS:-c2 c3}; do
  for v in old new old new; do
    cp abx/libs3imph_$v.so $L
    timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config $cfg --steps 20 \
      >> $OUT/${cfg}_$v.log 2>&1
  done
done
cp abx/libs3imph_new.so $L
# the new library once more per A/B knob setting (AB_ENV="S3IMPH_MID_FENCE=1 S3IMPH_SCAT_CFG=0": one run each)
i=0
for kv in $AB_ENV; do
  i=$((i+1))
  for cfg in c2 c3; do
    env $kv timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config $cfg --steps 20 \
      >> $OUT/${cfg}_knob${i}_${kv}.log 2>&1
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
