set -e
bash tools/gpu_round.sh r01s nopytest c2
mkdir -p gpurun_out/r01s
timeout -k 10 300 python bench.py --no-cpu-baseline --config c3 --steps 5 --warmup 1 > gpurun_out/r01s/bench_c3.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --config c5 --steps 5 --warmup 1 > gpurun_out/r01s/bench_c5.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --dist --steps 10 > gpurun_out/r01s/bench_dist1.log 2>&1
