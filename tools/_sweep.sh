set -e
mkdir -p gpurun_out/sw
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "hash_variants" > gpurun_out/sw/pytest.log 2>&1
for cfg in c2 c3; do
  for hm in 0 15; do
    S3IMPH_HASH_MODE=$hm timeout -k 10 120 python bench.py --no-cpu-baseline --config $cfg --steps 10 --warmup 2 > gpurun_out/sw/$cfg.hm$hm.log 2>&1
  done
done
S3IMPH_HASH_MODE=0 timeout -k 10 300 python tools/hash_probe.py > gpurun_out/sw/probe0.log 2>&1
S3IMPH_HASH_MODE=15 timeout -k 10 300 python tools/hash_probe.py > gpurun_out/sw/probe15.log 2>&1
