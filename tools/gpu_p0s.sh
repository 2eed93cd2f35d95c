#!/bin/bash
# S up to 64 (two 512-thread super-tile scatter blocks per CU): P0 parity subset, then C3 A/B
# of S3IMPH_P0_MAXS 64 / 32 (stage times)
OUT=gpurun_out/${1:-r4_p0s}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "p0 or big_tiles or c3_100m or c5_one_gpu or list_record or bitmap_level0" > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc $rc" >> $OUT/status; stop $rc; [ $rc = 0 ] || exit $rc
for rep in 1 2 3; do for v in 64 32; do
  S3IMPH_P0_MAXS=$v timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c3 --steps 20 >> $OUT/c3_maxs_$v.log 2>&1; rc=$?; stop $rc
done; done
S3IMPH_DEBUG=1 timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c3 --steps 2 --warmup 1 > $OUT/dbg.log 2>&1; rc=$?; stop $rc
python3 - > $OUT/summary.txt <<PY
import json, glob
for f in sorted(glob.glob("$OUT/c[23]_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d.get("stages_ms"))
PY
