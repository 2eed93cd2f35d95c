set -e
mkdir -p gpurun_out/sw
for cfg in c2 c3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --config $cfg --steps 30 --warmup 3 > gpurun_out/sw/$cfg.log 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/sw/pmc_write -o run -- python3 bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sw/pmcw.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/sw/pmc_fetch -o run -- python3 bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sw/pmcf.log 2>&1
