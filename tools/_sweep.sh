set -e
O=gpurun_out/hs
mkdir -p $O
for i in 1 2; do
  for k in 256 384 768; do
    S3IMPH_CHUNKS=$k timeout -k 10 120 python bench.py --no-cpu-baseline --config c2 --steps 20 --warmup 3 > $O/c2.ch$k.$i.log 2>&1
  done
  for m in 1 7 13; do
    S3IMPH_HASH_MODE=$m timeout -k 10 120 python bench.py --no-cpu-baseline --config c2 --steps 20 --warmup 3 > $O/c2.hm$m.$i.log 2>&1
  done
done
echo done > $O/DONE
