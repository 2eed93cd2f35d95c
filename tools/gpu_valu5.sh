#!/bin/bash
# VALU counters of the C5 build (skewed hash)
OUT=gpurun_out/${1:-r4_valu5}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $OUT/c5 -o run -- \
  python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --headline-only > $OUT/c5.log 2>&1 && \
S3IMPH_DEBUG=1 timeout -k 10 120 python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-secondary --headline-only > $OUT/c5_dbg.log 2>&1
echo "rc $?" > $OUT/status
