#!/bin/bash
# HBM traffic (FETCH_SIZE x2 / WRITE_SIZE, separate passes) of one build per config, merged
# into gpurun_out/TAG/pmc_traffic.json (copy to profiles/ to attach it to bench lines).
#   bash tools/gpu_pmc_all.sh TAG [configs...]
set -e
TAG=$1; shift
CFGS=${@:-c2 c3 c5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
for cfg in $CFGS; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_${ctr}_$cfg -o run -- \
      python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --headline-only \
      > $OUT/pmc_${ctr}_$cfg.log 2>&1
  done
  python3 tools/pmc_summary.py $OUT/pmc_FETCH_SIZE_$cfg/run_counter_collection.csv \
    $OUT/pmc_WRITE_SIZE_$cfg/run_counter_collection.csv $OUT/pmc_dispatches_$cfg.json $cfg $OUT/pmc_traffic.json \
    > $OUT/pmc_summary_$cfg.txt
done
echo done > $OUT/DONE
