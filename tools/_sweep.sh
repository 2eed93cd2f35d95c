set -e
mkdir -p gpurun_out/sw
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dist" > gpurun_out/sw/pytest.log 2>&1
timeout -k 10 120 python bench.py --no-cpu-baseline --dist --steps 30 --warmup 3 > gpurun_out/sw/dist.log 2>&1
