#!/bin/bash
# VALU counters of the level-0 hash (C3 bench, one build) and of the FNV microbenchmark
OUT=gpurun_out/${1:-r4_valu}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $OUT/c3 -o run -- \
  python3 bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --headline-only > $OUT/c3.log 2>&1 && \
timeout -s KILL 100 rocprofv3 --pmc $C --output-format csv -d $OUT/ub -o run -- ./tools/ubench_fnv_bin 4 > $OUT/ub.log 2>&1
echo "rc $?" > $OUT/status
