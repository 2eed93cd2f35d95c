set -e
mkdir -p gpurun_out/r01t
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dup or dist or golden or sizes or c2 or ragged" > gpurun_out/r01t/pytest.log 2>&1
for cfg in c2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --config $cfg --steps 20 --warmup 3 > gpurun_out/r01t/$cfg.log 2>&1
done
S3IMPH_DEBUG=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/r01t/c2dbg.log 2>&1
