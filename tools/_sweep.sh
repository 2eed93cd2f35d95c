set -e
mkdir -p gpurun_out/sw
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "lookup or c3 or dist or golden" > gpurun_out/sw/pytest.log 2>&1
for cfg in c2 c3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --config $cfg > gpurun_out/sw/$cfg.log 2>&1
done
