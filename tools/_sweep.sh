set -e
mkdir -p gpurun_out/sw
timeout -k 10 200 python bench.py > gpurun_out/sw/c2.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --dist > gpurun_out/sw/dist.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "profil or capi or stage or dist_host" > gpurun_out/sw/pytest.log 2>&1
