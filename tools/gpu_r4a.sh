#!/bin/bash
# dup probe, P0 + bitmap parity subset, C3 bench A/B of S3IMPH_P0, bitmap N=1 lanes A/B, C3 host phases
OUT=gpurun_out/r4_p0b; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
timeout -k 10 200 python tools/dup_probe.py > $OUT/probe.log 2>&1; rc=$?; echo "probe rc $rc" >> $OUT/status; stop $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  --durations=10 > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc $rc" >> $OUT/status; stop $rc
for rep in 1 2; do for cfg in c3 c2; do for v in 1 0; do
  S3IMPH_P0=$v timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config $cfg --steps 20 >> $OUT/${cfg}_p0_$v.log 2>&1; rc=$?; stop $rc
done; done; done
for v in planes counts; do
  S3IMPH_BM_LANES=$v timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c3 --steps 10 --dist --decomp bitmap >> $OUT/c3_bm_$v.log 2>&1; rc=$?; stop $rc
done
timeout -k 10 200 python tools/host_phase.py 100000000 64 --debug > $OUT/host_c3.log 2>&1; rc=$?; stop $rc
for m in 0 1 2; do
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$m -o run -- ./tools/ubench_fetch $m \
    > $OUT/fetch_$m.log 2>&1; rc=$?; stop $rc
done
python3 - > $OUT/summary.txt <<PY
import json, glob
for f in sorted(glob.glob("$OUT/c[23]_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d.get("stages_ms"))
PY
