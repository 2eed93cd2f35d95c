set -e
O=gpurun_out/pipe
mkdir -p $O
S3IMPH_PIPE0=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_pipe4.log 2>&1
for i in 1 2; do
for k in 0 2 4 8; do
  for cfg in c2 c3 c5; do
    S3IMPH_PIPE0=$k timeout -k 10 120 python bench.py --no-cpu-baseline --config $cfg --steps 20 --warmup 3 > $O/$cfg.k$k.$i.log 2>&1
  done
done
done
echo done > $O/DONE
