set -e
mkdir -p gpurun_out/sw
for cfg in c2 c3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --config $cfg > gpurun_out/sw/$cfg.log 2>&1
done
