#!/bin/bash
# GPU-box pass over the other bench configurations (C2, C4, C5, the multi-GPU path at
# N=1 on C2), the driver's smoke(), and C2's two HBM PMC passes; one bench line per
# config under gpurun_out/TAG.   bash tools/gpu_configs.sh TAG
set -e
TAG=${1:-cfg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
for cfg in c2 c4 c5; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --config $cfg --steps 10 --warmup 2 > $OUT/bench_$cfg.log 2>&1
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --config c2 --dist --steps 20 --warmup 3 > $OUT/bench_dist1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_c2 -o run -- \
  python3 bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/pmc_fetch_c2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_c2 -o run -- \
  python3 bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/pmc_write_c2.log 2>&1
echo done > $OUT/DONE
