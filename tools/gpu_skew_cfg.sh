#!/bin/bash
# k_hash_skew block / group shapes on C5 (S3IMPH_SKEW_CFG: 2 = 768 thr / 5120 keys (default), 1 = 1024 /
# 4096, 0 = 2 x 512 / 2048): parity of each, then alternating C5 bench runs.
#   bash tools/gpu_skew_cfg.sh TAG "2 1"
set -e
OUT=gpurun_out/$1; mkdir -p $OUT
CF=${2:-"2 1"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in $CF; do
  S3IMPH_SKEW_CFG=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -x -q \
    -k "c5_one_gpu or long_keys or level0_ragged or mixed" --timeout 200 --timeout-method thread > $OUT/pytest_cfg$c.log 2>&1
done
for rep in 1 2; do
  for c in $CF; do
    S3IMPH_SKEW_CFG=$c timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config c5 \
      --steps 10 --warmup 2 >> $OUT/c5_cfg$c.log 2>&1
  done
done
python3 - > $OUT/summary.txt <<PY
import json, glob
for f in sorted(glob.glob("$OUT/c5_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d.get("stages_ms"))
PY
echo done > $OUT/DONE
