#!/bin/bash
# The N > 1 bench path on the one-GPU box: `bench.py --gpus 2` launches its own 2 ranks (gloo process group,
# both ranks on the one device), weak scaling, max-over-ranks clock, the statistics all-reduce.
set -o pipefail
OUT=${1:-gpurun_out/rehearsal2}
mkdir -p "$OUT"
RMX_BENCH_BACKEND=gloo timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 200 --warmup 20 --large-envs 0 \
  --no-cpu-baseline --no-rollout > "$OUT/bench_gpus2.json" 2> "$OUT/bench_gpus2.err" || { tail -20 "$OUT/bench_gpus2.err"; exit 1; }
cat "$OUT/bench_gpus2.json"
