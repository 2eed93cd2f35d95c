set -e
O=gpurun_out/hs2
mkdir -p $O
for i in 1 2; do
  for m in 3 7; do
    S3IMPH_HASH_MODE=$m timeout -k 10 120 python bench.py --no-cpu-baseline --config c2 --steps 20 --warmup 3 > $O/c2.hm$m.$i.log 2>&1
    S3IMPH_HASH_MODE=$m timeout -k 10 120 python bench.py --no-cpu-baseline --config c3 --steps 10 --warmup 2 > $O/c3.hm$m.$i.log 2>&1
  done
done
echo done > $O/DONE
