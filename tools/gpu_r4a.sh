#!/bin/bash
# dup probe, P0 parity subset, C3 bench A/B of S3IMPH_P0
OUT=gpurun_out/r4_p0b; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python tools/dup_probe.py > $OUT/probe.log 2>&1; rc=$?
echo "probe rc $rc" >> $OUT/status
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "p0 or big_tiles or c3_100m_bit_exact or c5_one_gpu_share" > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc $rc" >> $OUT/status
case $rc in 124|134|137|139) exit $rc;; esac
for rep in 1 2; do for v in 1 0; do
  S3IMPH_P0=$v timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c3 --steps 20 >> $OUT/c3_$v.log 2>&1 || exit $?
done; done
python3 - > $OUT/summary.txt <<PY
import json, glob
for f in sorted(glob.glob("$OUT/c*_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d.get("stages_ms"))
PY
