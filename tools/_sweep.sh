set -e
mkdir -p gpurun_out/sw
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "hash_variants or counted_path or overflow_reruns or direct_scatter" > gpurun_out/sw/pytest.log 2>&1
