#!/bin/bash
# Kernel-trace + PMC passes of bench.py on the GPU box (run from the repo root via gpurun).
# Counters are collected in their own passes (no sys/runtime trace alongside --pmc).
#   bash scripts/profile.sh OUTDIR ["bench.py args"]
set -o pipefail
OUT=${1:-gpurun_out/prof}
ARGS=${2:-"--no-cpu-baseline --no-rollout --large-envs 0 --steps 1000 --warmup 100"}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 bench.py $ARGS > "$OUT/kt_bench.json" 2> "$OUT/kt.err" || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o pmc -- python3 bench.py $ARGS --graph 0 > "$OUT/pmc_$c.json" 2> "$OUT/pmc_$c.err" || exit $?
done
