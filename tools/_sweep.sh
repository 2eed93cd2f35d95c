set -e
mkdir -p gpurun_out/sw
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "hash_variants" > gpurun_out/sw/pytest.log 2>&1
for cfg in c5 c2; do
  for hm in 0 18; do
    S3IMPH_HASH_MODE=$hm timeout -k 10 120 python bench.py --no-cpu-baseline --config $cfg --steps 20 --warmup 3 > gpurun_out/sw/$cfg.hm$hm.log 2>&1
  done
done
