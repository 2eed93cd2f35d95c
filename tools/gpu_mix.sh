#!/bin/bash
# ubench + selected GPU tests
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 60 ./tools/ubench_fnv.bin > $OUT/ubench_fnv.txt 2>&1
timeout -k 10 800 python -u -m pytest ${2:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo done > $OUT/DONE
