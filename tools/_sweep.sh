set -e
O=gpurun_out/ch2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
for i in 1 2; do
  for cfg in c2 c3 c4 c5; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --config $cfg --steps 20 --warmup 3 > $O/$cfg.$i.log 2>&1
  done
done
echo done > $O/DONE
