#!/bin/bash
# Round-3 characterisation at the tree: r03h (config-3 table modes / block sizes, lookup ablations, in-kernel
# stamps of configs 3 and 2, slip fast vs generic, floor_bench under the tracer with graphs kept alive), then
# FrozenLake random starts (generic kernel) beside the deterministic fast kernel, and one bench line of the
# four GPU configs with the 500-step chain time beside the window time.
set -o pipefail
OUT=${OUT:-gpurun_out/r03k}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --large-envs 0 --dict-seconds 0 \
  --no-rollout > $OUT/bench_chain.json 2> $OUT/bench_chain.err || { tail -20 $OUT/bench_chain.err; exit 1; }
timeout -k 10 300 python -u scripts/variants.py --random-starts 1 --configs 2,4 --variants fast:64,tpe:256,tpe:64 --rollout 1 > $OUT/randstart.log 2>&1 || { tail -20 $OUT/randstart.log; exit 1; }
cat $OUT/randstart.log
OUT=$OUT bash scripts/gpu_r03h.sh
