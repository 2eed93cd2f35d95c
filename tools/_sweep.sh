set -e
O=gpurun_out/tail2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
for i in 1 2 3; do
  for cfg in c2 c5; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --config $cfg --steps 20 --warmup 3 > $O/$cfg.$i.log 2>&1
  done
done
timeout -k 10 300 python -u tools/tile_phase_probe.py > $O/tp_c2.log 2>&1
timeout -k 10 400 python -u tools/flake_probe.py 40 10000000 > $O/flake.log 2>&1
echo done > $O/DONE
