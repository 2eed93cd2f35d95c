#!/bin/bash
set -e
TAG=${1:-r3f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ragged or c5 or skew or unbalanced or sizes" > $OUT/pytest_gpu.log 2>&1
S3IMPH_SKEW_CFG=2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "c5_one_gpu_share or ragged or skew" > $OUT/pytest_gpu_cfg2.log 2>&1
B="python bench.py --no-cpu-baseline --no-secondary --headline-only"
for cfg in 1 2; do export S3IMPH_SKEW_CFG=$cfg;
  timeout -k 10 300 $B --config c5 --steps 10 --warmup 2 > $OUT/c5_cfg$cfg.log 2>&1
  timeout -k 10 300 python tools/skew_phase.py > $OUT/skew_phase_cfg$cfg.log 2>&1
done
echo done > $OUT/DONE
