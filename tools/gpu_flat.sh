#!/bin/bash
# flat dword write phase of the super-tile scatter: P0 parity subset, C3 A/B of S3IMPH_P0_FLAT
# (and S3IMPH_P0_MAXS 64 / 32 with it), PMC of the scatter
OUT=gpurun_out/${1:-r4_flat}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "p0 or big_tiles or c3_100m or c5_one_gpu or bitmap_level0" > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc $rc" >> $OUT/status; stop $rc; [ $rc = 0 ] || exit $rc
for rep in 1 2 3; do for v in "1 64" "0 64" "1 32" "0 32"; do set -- $v
  S3IMPH_P0_FLAT=$1 S3IMPH_P0_MAXS=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c3 --steps 20 >> $OUT/c3_flat$1_s$2.log 2>&1; rc=$?; stop $rc
done; done
python3 - > $OUT/summary.txt <<PY
import json, glob
for f in sorted(glob.glob("$OUT/c[23]_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d.get("stages_ms"))
PY
