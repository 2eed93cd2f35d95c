set -e
mkdir -p gpurun_out/r01t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "direct or big_tiles or c3 or c2 or level0 or golden or dist_host" > gpurun_out/r01t/pytest.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r01t/c2.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --config c3 --steps 10 --warmup 2 > gpurun_out/r01t/c3.log 2>&1
S3IMPH_DEBUG=1 timeout -k 10 200 python bench.py --no-cpu-baseline --config c3 --steps 1 --warmup 1 > gpurun_out/r01t/c3dbg.log 2>&1
