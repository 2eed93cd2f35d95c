#!/bin/bash
# One GPU-box step, run through gpurun from the repo root.  Every step writes under
# gpurun_out/TAG/ and runs under its own time limit; chain steps with && so a failed
# or timed-out step ends the call.
#
#   bash tools/gpu.sh TAG pytest [-k EXPR]        the -m gpu suite (per-test timeout) -> pytest_gpu.log
#   bash tools/gpu.sh TAG bench NAME [bench args]  one bench.py line -> NAME.log
#   bash tools/gpu.sh TAG prof NAME [bench args]   rocprofv3 --kernel-trace --stats of a short bench run
#                                                 -> NAME/ (csv), NAME_stats.csv, NAME_timeline.txt
#   bash tools/gpu.sh TAG pmc NAME CFG [bench args] FETCH_SIZE and WRITE_SIZE passes (one run each) of one
#                                                 build, summarised per kernel into pmc_NAME.txt and
#                                                 merged into gpurun_out/TAG/pmc_traffic.json
#   bash tools/gpu.sh TAG ctr NAME "CTRS" [bench args]
#                                                 one rocprofv3 --pmc pass with the given counters (at
#                                                 most 8 SQ_ / 4 TCC_ / 2 GRBM_ ...) over one build -> NAME/
#   bash tools/gpu.sh TAG ab REPS CFG "ENV_A" "ENV_B" ...
#                                                 env-knob A/B on one config, alternating (each ENV a list
#                                                 of VAR=VALUE, "-" for none; S3IMPH_DEV=1 is implied so
#                                                 the library reads the dev knobs) -> ab_summary.txt
#   bash tools/gpu.sh TAG lib REPS CFG            old / new library A/B (abx/libs3imph_{old,new}.so,
#                                                 alternating) -> lib_summary.txt
#   bash tools/gpu.sh TAG host NAME [args]        tools/host_phase.py (host-memory build phases) -> NAME.log
#   bash tools/gpu.sh TAG hostab REPS N AVG "ENV_A" "ENV_B" ...
#                                                 env-knob A/B of the same, alternating -> hostab.log
#   bash tools/gpu.sh TAG p8 NAME [P K AVG BUILDS]
#                                                 tools/p8_geometry.py under rocprofv3 --kernel-trace: the
#                                                 P-rank bitmap build on this one GPU, ranks serialised; per-
#                                                 rank kernel sums -> NAME_ranks.txt
#   bash tools/gpu.sh TAG multi NAME NPROC [bench args]
#                                                 bench.py's N > 1 path under torchrun, ranks sharing
#                                                 this one GPU through the host transport -> NAME.log
# BENCH_EXTRA is appended to every bench.py command line.
set -o pipefail
TAG=$1; STEP=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
short="--steps 5 --warmup 2 --no-cpu-baseline --no-secondary --headline-only"
stop() {  # a GPU fault, abort, segfault or time limit ends the whole call
  case $1 in 124|134|137|139) echo "$STEP stopped rc $1" >> "$OUT/status"; exit "$1";; esac
  return 0
}
case $STEP in
  pytest)
    K=()
    [ "$1" = "-k" ] && K=(-k "$2")
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 400 --timeout-method thread \
      "${K[@]}" > "$OUT/pytest_gpu.log" 2>&1
    rc=$?; echo "pytest rc $rc" >> "$OUT/status"; exit $rc ;;
  bench)
    NAME=$1; shift
    timeout -k 10 500 python bench.py "$@" $BENCH_EXTRA > "$OUT/$NAME.log" 2>&1
    rc=$?; echo "bench $NAME rc $rc" >> "$OUT/status"; exit $rc ;;
  prof)
    NAME=$1; shift
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$NAME" -o run -- \
      python3 bench.py $short "$@" $BENCH_EXTRA > "$OUT/${NAME}_bench.log" 2>&1
    rc=$?; stop $rc
    cp "$OUT/$NAME/run_kernel_stats.csv" "$OUT/${NAME}_stats.csv" 2>/dev/null
    python3 tools/trace_summary.py "$OUT/$NAME/run_kernel_trace.csv" 0 > "$OUT/${NAME}_timeline.txt"
    echo "prof $NAME rc $rc" >> "$OUT/status"; exit $rc ;;
  pmc)
    NAME=$1; CFG=$2; shift 2
    [ -f "$OUT/pmc_traffic.json" ] || cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_${ctr}_$NAME" -o run -- \
        python3 bench.py --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --headline-only \
        "$@" $BENCH_EXTRA > "$OUT/pmc_${ctr}_$NAME.log" 2>&1
      rc=$?; stop $rc
      [ $rc = 0 ] || exit $rc
    done
    python3 tools/pmc_summary.py "$OUT/pmc_FETCH_SIZE_$NAME/run_counter_collection.csv" \
      "$OUT/pmc_WRITE_SIZE_$NAME/run_counter_collection.csv" "$OUT/pmc_dispatches_$NAME.json" "$NAME" \
      "$OUT/pmc_traffic.json" > "$OUT/pmc_$NAME.txt"
    echo "pmc $NAME rc $?" >> "$OUT/status" ;;
  ctr)
    NAME=$1; CTRS=$2; shift 2
    timeout -s KILL 150 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/$NAME" -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --headline-only "$@" $BENCH_EXTRA \
      > "$OUT/$NAME.log" 2>&1
    rc=$?; echo "ctr $NAME rc $rc" >> "$OUT/status"; exit $rc ;;
  ab)
    REPS=$1; CFG=$2; shift 2
    for rep in $(seq "$REPS"); do
      i=0
      for e in "$@"; do
        i=$((i+1)); envs="S3IMPH_DEV=1"; [ "$e" != "-" ] && envs="$envs $e"
        env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config "$CFG" \
          --steps 20 $BENCH_EXTRA >> "$OUT/ab_v$i.log" 2>&1
        rc=$?; echo "ab v$i ($e) rep $rep rc $rc" >> "$OUT/status"; stop $rc
      done
    done
    python3 tools/ab_summary.py "$OUT" ab "$@" > "$OUT/ab_summary.txt" ;;
  lib)
    REPS=$1; CFG=$2
    L=s3-inv-db_amd/s3imph/_lib/libs3imph.so
    for rep in $(seq "$REPS"); do
      for v in old new; do
        cp "abx/libs3imph_$v.so" $L
        timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --no-secondary --config "$CFG" --steps 20 \
          $BENCH_EXTRA >> "$OUT/lib_${CFG}_$v.log" 2>&1
        rc=$?; echo "lib $v rep $rep rc $rc" >> "$OUT/status"; stop $rc
      done
    done
    cp abx/libs3imph_new.so $L
    python3 tools/ab_summary.py "$OUT" "lib_${CFG}" old new > "$OUT/lib_${CFG}_summary.txt" ;;
  hostab)
    # env-knob A/B of the host-memory build (tools/host_phase.py --phases), alternating
    REPS=$1; N=$2; AVG=$3; shift 3
    for rep in $(seq "$REPS"); do
      i=0
      for e in "$@"; do
        i=$((i+1)); envs="S3IMPH_DEV=1"; [ "$e" != "-" ] && envs="$envs $e"
        echo "== v$i ($e) rep $rep" >> "$OUT/hostab.log"
        env $envs timeout -k 10 200 python tools/host_phase.py "$N" "$AVG" --phases >> "$OUT/hostab.log" 2>&1
        rc=$?; echo "hostab v$i ($e) rep $rep rc $rc" >> "$OUT/status"; stop $rc
      done
    done ;;
  host)
    NAME=$1; shift
    timeout -k 10 300 python tools/host_phase.py "$@" > "$OUT/$NAME.log" 2>&1
    rc=$?; echo "host $NAME rc $rc" >> "$OUT/status"; exit $rc ;;
  p8)
    NAME=$1; shift
    timeout -k 10 1000 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$NAME" -o run -- \
      python3 tools/p8_geometry.py "$@" > "$OUT/$NAME.log" 2>&1
    rc=$?; stop $rc
    python3 tools/rank_kernel_sums.py "$OUT/$NAME/run_kernel_trace.csv" > "$OUT/${NAME}_ranks.txt"
    echo "p8 $NAME rc $rc" >> "$OUT/status"; exit $rc ;;
  multi)
    NAME=$1; NP=$2; shift 2
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NP" --master-addr 127.0.0.1 \
      --master-port 29541 bench.py --gpus "$NP" --transport host "$@" $BENCH_EXTRA > "$OUT/$NAME.log" 2>&1
    rc=$?; echo "multi $NAME rc $rc" >> "$OUT/status"; exit $rc ;;
  *)
    echo "unknown step $STEP" >&2; exit 2 ;;
esac
