set -e
mkdir -p gpurun_out/sw
timeout -k 10 300 python -u tools/flake_probe.py 100 300000 > gpurun_out/sw/flake300k.log 2>&1
timeout -k 10 300 python -u tools/flake_probe.py 60 2500000 > gpurun_out/sw/flake2m5.log 2>&1
timeout -k 10 300 python -u tools/flake_probe.py 30 25000000 > gpurun_out/sw/flake25m.log 2>&1
