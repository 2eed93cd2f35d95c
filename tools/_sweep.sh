set -e
mkdir -p gpurun_out/sw
for i in 1 2; do
for w in 0 1; do
  for cfg in c2 c5; do
    S3IMPH_TILE_WIDE=$w timeout -k 10 120 python bench.py --no-cpu-baseline --config $cfg --steps 30 --warmup 3 > gpurun_out/sw/$cfg.w$w.$i.log 2>&1
  done
done
done
timeout -k 10 300 python -u tools/flake_probe.py 40 > gpurun_out/sw/flake.log 2>&1
