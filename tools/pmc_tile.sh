#!/bin/bash
# SQ counters of the split big-tile and reservation-scatter kernels on one C3 build, one pass each.
#   bash tools/pmc_tile.sh TAG [config]
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE"
for i in 1 2; do
  eval P=\"\$P$i\"
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 bench.py --config ${2:-c3} --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > $OUT/p$i.log 2>&1
done
for k in k_tile_split k_scatter_res; do
  echo "== $k"
  python3 tools/pmc_kernel.py $OUT/p1/run_counter_collection.csv $OUT/p2/run_counter_collection.csv -k $k -i 0
done > $OUT/summary.txt
echo done > $OUT/DONE
