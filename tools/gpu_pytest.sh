#!/bin/bash
# A -m gpu subset on the in-tree build:  bash tools/gpu_pytest.sh TAG "pytest -k expr" [test files...]
set -e
OUT=gpurun_out/$1; K=$2; shift 2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" \
  > $OUT/pytest.log 2>&1
echo done > $OUT/DONE
