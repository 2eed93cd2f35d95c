set -e
mkdir -p gpurun_out/sw
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sw/pytest.log 2>&1
for cfg in c2 c3 c5; do
  for r in 0 1; do
    S3IMPH_RES2=$r timeout -k 10 120 python bench.py --no-cpu-baseline --config $cfg --steps 20 --warmup 3 > gpurun_out/sw/$cfg.r$r.log 2>&1
  done
done
