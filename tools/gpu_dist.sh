set -e
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_multi.py tests/test_gpu_scale.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 200 python bench.py --dist --no-cpu-baseline --headline-only > $OUT/bench_dist_c3.log 2>&1
timeout -k 10 200 python bench.py --dist --config c2 --no-cpu-baseline --headline-only > $OUT/bench_dist_c2.log 2>&1
echo done > $OUT/DONE
