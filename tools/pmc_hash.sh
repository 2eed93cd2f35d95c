#!/bin/bash
# SQ counters of the level-0 hash kernels (and the FNV microbenchmark), one pass each.
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA"
timeout -s KILL 60 rocprofv3 --pmc $P1 --output-format csv -d $OUT/ub1 -o run -- ./tools/ubench_fnv.bin > $OUT/ub1.log 2>&1
for h in 0 1; do
  S3IMPH_H0=$h timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $OUT/h${h}_p1 -o run -- python3 bench.py --config ${2:-c3} --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/h${h}_p1.log 2>&1
  S3IMPH_H0=$h timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d $OUT/h${h}_p2 -o run -- python3 bench.py --config ${2:-c3} --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/h${h}_p2.log 2>&1
done
echo done > $OUT/DONE
