set -e
mkdir -p gpurun_out/r01r
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01r/pytest.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r01r/c2.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1 > gpurun_out/r01r/c3.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --config c5 --steps 5 --warmup 1 > gpurun_out/r01r/c5.log 2>&1
