set -e
mkdir -p gpurun_out/sweep1
run() { tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sweep1/$tag.log 2>&1; }
run base
run t0_4096 S3IMPH_TARGET_TILES0=4096
run tl_2048 S3IMPH_TARGET_TILES=2048
run tl_512 S3IMPH_TARGET_TILES=512
run res_512 S3IMPH_TARGET_TILES_RES=512
run res_1024 S3IMPH_TARGET_TILES_RES=1024
run resmax_4m S3IMPH_RES_MAX=4500000
