#!/bin/bash
# rocprofv3 evidence of the default step kernel at HEAD, per BASELINE config (65,536 envs) and at the
# HBM-resident size (config 2 shape, 8,388,608 envs): one --kernel-trace --stats pass of bench.py, then
# FETCH_SIZE and WRITE_SIZE in passes of their own.  All passes use --graph 0 (eager launches): traced inside a
# replayed HIP graph the step kernel's dispatches read ~4.1-4.8 us (the tracer's per-dispatch handling), traced
# eagerly they read 3.2 us, the live per-launch time of the graph-replayed bench (r02af).
#   bash scripts/profile_configs.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/profcfg}
export TMPDIR=/tmp
mkdir -p "$OUT"
run() {  # name, bench args
  local d="$OUT/$1"; shift
  mkdir -p "$d"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d/kt" -o kt -- \
    python3 bench.py "$@" --graph 0 --spin-ms 50 > "$d/kt_bench.json" 2> "$d/kt.err" || { tail -5 "$d/kt.err"; return 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$d/pmc_$c" -o pmc -- \
      python3 bench.py "$@" --graph 0 --steps 100 --warmup 10 --windows 1 --spin-ms 0 > "$d/pmc_$c.json" 2> "$d/pmc_$c.err" \
      || { tail -5 "$d/pmc_$c.err"; return 1; }
  done
  echo "profiled $d"
}
COMMON="--no-cpu-baseline --no-rollout --large-envs 0 --dict-seconds 0"
for c in ${CFGS:-2 3 4 5 hbm slip2 slip3}; do  # CFGS="hbm" (say) profiles a subset
  if [ "$c" = hbm ]; then
    run hbm --config 2 $COMMON --n-envs 8388608 --steps 50 --warmup 5 --windows 2 || exit 1
  elif [ "${c#slip}" != "$c" ]; then  # slip2 / slip3: the config with its env's slip switch on (bench.py --slip)
    run $c --config ${c#slip} --slip $COMMON --steps 200 --warmup 10 --windows 2 || exit 1
  else
    run cfg$c --config $c $COMMON --steps 200 --warmup 10 --windows 2 || exit 1
  fi
done
