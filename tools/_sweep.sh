set -e
mkdir -p gpurun_out/sw
for cfg in c2 c3 c5; do
  for rm in 2097152 8388608 16777216 50331648; do
    S3IMPH_RES_MAX=$rm S3IMPH_RES_FILL=2 timeout -k 10 120 python bench.py --no-cpu-baseline --config $cfg --steps 20 --warmup 3 > gpurun_out/sw/$cfg.res$rm.log 2>&1
  done
done
