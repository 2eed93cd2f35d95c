set -e
mkdir -p gpurun_out/sw
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sw/pytest.log 2>&1
