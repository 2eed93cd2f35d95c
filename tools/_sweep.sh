set -e
mkdir -p gpurun_out/sw
for t0 in 2048 4096; do
  for t in 1024 2048; do
    S3IMPH_TARGET_TILES0=$t0 S3IMPH_TARGET_TILES=$t timeout -k 10 120 python bench.py --no-cpu-baseline --config c2 --steps 30 --warmup 3 > gpurun_out/sw/c2.t$t0.$t.log 2>&1
  done
done
for tr in 128 256 512; do
  S3IMPH_TARGET_TILES_RES=$tr timeout -k 10 120 python bench.py --no-cpu-baseline --config c2 --steps 30 --warmup 3 > gpurun_out/sw/c2.tr$tr.log 2>&1
done
