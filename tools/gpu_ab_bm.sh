#!/bin/bash
# bitmap-decomposition A/B of two libraries (abx/libs3imph_{old,new}.so, alternating) on C3 N=1,
# after the multi / dist GPU tests on the new one.   bash tools/gpu_ab_bm.sh TAG
OUT=gpurun_out/${1:-r4_abbm}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
L=s3-inv-db_amd/s3imph/_lib/libs3imph.so
cp abx/libs3imph_new.so $L
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_dist.py -m gpu -x -v --timeout 400 \
  --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc $rc" >> $OUT/status; stop $rc; [ $rc = 0 ] || exit $rc
for rep in 1 2 3; do for v in old new; do
  cp abx/libs3imph_$v.so $L
  timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c3 --steps 10 --warmup 2 --dist --decomp bitmap >> $OUT/bm_$v.log 2>&1; rc=$?; stop $rc
done; done
cp abx/libs3imph_new.so $L
python3 - > $OUT/summary.txt <<PY
import json, glob
for f in sorted(glob.glob("$OUT/bm_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d.get("stages_ms"))
PY
