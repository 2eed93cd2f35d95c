#!/bin/bash
# bench.py's N > 1 code path (torchrun, one process per rank, gloo for the timing
# reductions) on ONE GPU: ranks share the device and exchange through the host-copy
# transport instead of RCCL.  A functional check of the multi-rank bench line; the
# numbers are not a scaling measurement.   bash tools/gpu_bench_multi_host.sh TAG
set -e
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --config c2 --transport host --steps 5 --warmup 2 --no-cpu-baseline \
  > $OUT/bench_n2_c2_host.log 2>&1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29532 bench.py --gpus 2 --config c3 --transport host --steps 3 --warmup 1 --no-cpu-baseline \
  > $OUT/bench_n2_c3_host.log 2>&1
echo done > $OUT/DONE
