#!/bin/bash
# The one launcher for GPU-box work (run from the repo root through gpurun).  ONE step per invocation, each under
# its own time limit; chain steps with && in the gpurun command so that the first failure ends the call.
#
#   bash scripts/gpu.sh smoke    OUT
#   bash scripts/gpu.sh tests    OUT TAG [pytest args ...]        -m gpu suite (or a -k subset) -> OUT/tests_TAG.txt
#   bash scripts/gpu.sh bench    OUT TAG [bench.py args ...]      -> OUT/bench_TAG.json (+ .err)
#   bash scripts/gpu.sh variants OUT TAG [variants.py args ...]   -> OUT/var_TAG.log
#   bash scripts/gpu.sh libs     OUT TAG "a.so b.so" [variants.py args ...]
#                                same-box A/B: the libraries alternated REPS (3) times -> OUT/libs_TAG.log
#   bash scripts/gpu.sh ktrace   OUT TAG [bench.py args ...]      rocprofv3 --kernel-trace --stats of bench.py
#   bash scripts/gpu.sh pmc      OUT TAG "COUNTERS" [bench.py args ...]   one --pmc pass of bench.py
#   bash scripts/gpu.sh profile  OUT TAG [bench.py args ...]      ktrace + FETCH_SIZE + WRITE_SIZE passes
#   bash scripts/gpu.sh floor    OUT TAG [floor_bench args ...]   scripts/floor_bench (built here with make -C scripts)
#   bash scripts/gpu.sh twtrace  OUT TAG CONFIG [trace_window.py args ...]
#                                K-step queue windows (scripts/trace_window.py) untraced, then under
#                                rocprofv3 --kernel-trace --stats -> OUT/TAG/{tw_notrace.json, tw.json, kt/}
#
# Every rocprofv3 pass runs eager HIP launches (--graph 0 --dispatch graph): traced inside a replayed HIP graph the
# step kernel's dispatches read 4.1-4.8 us, traced through the engine's own queue (rmx_step_seq, the tracer's queue
# interception) 4.15 us (r04x), traced eagerly they agree with the live per-launch time of the bench.
# Counter passes hold one block's counters only (no trace domains).
set -o pipefail
export TMPDIR=/tmp
kind=$1 OUT=$2
shift 2 || { echo "usage: bash scripts/gpu.sh KIND OUT [TAG] [args]"; exit 2; }
mkdir -p "$OUT"
fail() { echo "gpu.sh $kind $TAG: exit $1"; tail -${2:-30} "$3"; exit "$1"; }
PROF_BENCH="--graph 0 --dispatch graph --spin-ms 50 --no-cpu-baseline --no-rollout --large-envs 0 --dict-seconds 0 --rs-configs="
case $kind in
  smoke)
    TAG=smoke
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || fail $? 30 "$OUT/smoke.log"
    tail -1 "$OUT/smoke.log" ;;
  tests)
    TAG=$1; shift
    timeout -k 10 1100 python -u -m pytest tests -m gpu -q --durations=25 --timeout 300 --timeout-method thread "$@" \
      > "$OUT/tests_$TAG.txt" 2>&1 || fail $? 40 "$OUT/tests_$TAG.txt"
    tail -2 "$OUT/tests_$TAG.txt" ;;
  bench)
    TAG=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || fail $? 30 "$OUT/bench_$TAG.err"
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', sys.argv[2], round(d['value']/1e9, 2), 'G/s', \
round(d['us_per_step_event'], 3), 'us/step (events)')" "$OUT/bench_$TAG.json" "$TAG" ;;
  variants)
    TAG=$1; shift
    timeout -k 10 400 python -u scripts/variants.py "$@" > "$OUT/var_$TAG.log" 2>&1 || fail $? 30 "$OUT/var_$TAG.log"
    grep '^{' "$OUT/var_$TAG.log" ;;
  libs)
    TAG=$1 LIBS=$2; shift 2
    for rep in $(seq 1 ${REPS:-3}); do
      for lib in $LIBS; do
        RMX_LIB=$lib timeout -k 10 300 python -u scripts/variants.py --rollout 0 "$@" > "$OUT/libs_one.log" 2>&1 \
          || fail $? 30 "$OUT/libs_one.log"
        grep '^{' "$OUT/libs_one.log" | sed "s|^|$(basename "$lib") rep=$rep |"
      done
    done | tee "$OUT/libs_$TAG.log" ;;
  ktrace)
    TAG=$1; shift
    d="$OUT/$TAG"; mkdir -p "$d"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d/kt" -o kt -- \
      python3 bench.py $PROF_BENCH "$@" > "$d/kt_bench.json" 2> "$d/kt.err" || fail $? 10 "$d/kt.err"
    echo "ktrace $d" ;;
  pmc)
    TAG=$1 CTRS=$2; shift 2
    d="$OUT/$TAG"; mkdir -p "$d"
    timeout -s KILL 180 rocprofv3 --pmc $CTRS --output-format csv -d "$d/pmc_${CTRS// /_}" -o pmc -- \
      python3 bench.py $PROF_BENCH --windows 1 --spin-ms 0 --chain 0 "$@" > "$d/pmc.json" 2> "$d/pmc.err" \
      || fail $? 10 "$d/pmc.err"
    echo "pmc $d $CTRS" ;;
  profile)
    TAG=$1; shift
    bash "$0" ktrace "$OUT" "$TAG" "$@" && bash "$0" pmc "$OUT" "$TAG" FETCH_SIZE "$@" && \
      bash "$0" pmc "$OUT" "$TAG" WRITE_SIZE "$@" || exit $? ;;
  twtrace)
    TAG=$1 CFG=$2; shift 2
    d="$OUT/$TAG"; mkdir -p "$d"
    timeout -k 10 120 python3 scripts/trace_window.py --config "$CFG" "$@" > "$d/tw_notrace.json" 2> "$d/tw_notrace.err" \
      || fail $? 10 "$d/tw_notrace.err"
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$d/kt" -o kt -- \
      python3 scripts/trace_window.py --config "$CFG" "$@" > "$d/tw.json" 2> "$d/tw.err" || fail $? 10 "$d/tw.err"
    echo "twtrace $d $(cat "$d/tw_notrace.json")" ;;
  floor)
    TAG=$1; shift
    timeout -k 10 300 ./scripts/floor_bench "$@" > "$OUT/floor_$TAG.log" 2>&1 || fail $? 20 "$OUT/floor_$TAG.log"
    cat "$OUT/floor_$TAG.log" ;;
  *) echo "gpu.sh: unknown step $kind"; exit 2 ;;
esac
