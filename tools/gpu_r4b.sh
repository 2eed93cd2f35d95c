#!/bin/bash
# P0 parity subset, then C3 / C2 A/B of S3IMPH_P0 (stage times), one timeline of C3
OUT=gpurun_out/r4_p0f; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
stop() { case $1 in 124|134|137|139) echo "stopped rc $1" >> $OUT/status; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  -k "p0 or big_tiles or c3_100m_bit_exact or c5_one_gpu_share or c4_one_gpu_share or dup or repeated_builds" > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc $rc" >> $OUT/status; stop $rc
for rep in 1 2; do for cfg in c3; do for v in 1 0; do
  S3IMPH_P0=$v timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config $cfg --steps 20 >> $OUT/${cfg}_p0_$v.log 2>&1; rc=$?; stop $rc
done; done; done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_c3 -o run -- \
  python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --headline-only > $OUT/prof_c3.log 2>&1; rc=$?; stop $rc
python3 tools/trace_summary.py $OUT/prof_c3/run_kernel_trace.csv 0 > $OUT/timeline_c3.txt
python3 - > $OUT/summary.txt <<PY
import json, glob
for f in sorted(glob.glob("$OUT/c[23]_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d.get("stages_ms"))
PY
S3IMPH_DEBUG=1 S3IMPH_P0=1 timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c3 --steps 2 --warmup 1 > $OUT/dbg_p0_1.log 2>&1; rc=$?; stop $rc
