#!/bin/bash
# SQ / memory counters of the isolated level-0 hash (tools/hash_only.py), one pass each.
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="FETCH_SIZE"
P3="WRITE_SIZE"
P4="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA"
for h in ${2:-0}; do
  for i in ${PASSES:-1 2 3 4}; do
    eval P=\"\$P$i\"
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/h${h}_p$i -o run -- python3 tools/hash_only.py ${3:-c3} 2 > $OUT/h${h}_p$i.log 2>&1
  done
done
echo done > $OUT/DONE
