set -e
mkdir -p gpurun_out/sw
for cfg in c2 c3 c5; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --config $cfg --steps 20 --warmup 3 > gpurun_out/sw/$cfg.log 2>&1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sw/pytest.log 2>&1
