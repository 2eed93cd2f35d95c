set -e
mkdir -p gpurun_out/sw
for i in 1 2; do
for cfg in c2 c3; do
  for hm in 0 17; do
    S3IMPH_HASH_MODE=$hm timeout -k 10 120 python bench.py --no-cpu-baseline --config $cfg --steps 20 --warmup 3 > gpurun_out/sw/$cfg.hm$hm.$i.log 2>&1
  done
done
done
