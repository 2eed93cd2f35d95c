set -e
O=gpurun_out/k1
mkdir -p $O
for i in 1 2; do
for k in 0 1; do
  for cfg in c2 c3 c4; do
    S3IMPH_PIPE0=$k timeout -k 10 120 python bench.py --no-cpu-baseline --config $cfg --steps 20 --warmup 3 > $O/$cfg.k$k.$i.log 2>&1
  done
done
done
echo done > $O/DONE
