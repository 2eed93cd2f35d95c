set -e
mkdir -p gpurun_out
run() { tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 200 python tools/c3_debug.py 10000000 32 > gpurun_out/tprof_a.log 2>&1
run a
run b S3IMPH_CHUNKS=512
run c S3IMPH_TARGET_TILES_RES=512
run d S3IMPH_TARGET_TILES_RES=128
