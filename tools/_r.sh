set -e
mkdir -p gpurun_out/r01t
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01t/pytest.log 2>&1
for cfg in c2 c3 c5; do
timeout -k 10 200 python bench.py --no-cpu-baseline --config $cfg --steps 20 --warmup 3 > gpurun_out/r01t/$cfg.log 2>&1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --dist --steps 20 --warmup 3 > gpurun_out/r01t/dist.log 2>&1
