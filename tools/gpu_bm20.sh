#!/bin/bash
# R20 list levels in the bitmap decomposition: multi / dist GPU tests, then C3 N=1 bitmap A/B of S3IMPH_L20
OUT=gpurun_out/${1:-r4_bm20}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_dist.py tests/test_gpu_scale.py -m gpu -x -v --timeout 400 \
  --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc $rc" >> $OUT/status; stop $rc; [ $rc = 0 ] || exit $rc
for rep in 1 2 3; do for v in 1 0; do
  S3IMPH_L20=$v timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c3 --steps 10 --warmup 2 --dist --decomp bitmap >> $OUT/bm_l20_$v.log 2>&1; rc=$?; stop $rc
done; done
python3 - > $OUT/summary.txt <<PY
import json, glob
for f in sorted(glob.glob("$OUT/bm_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d.get("stages_ms"))
PY
