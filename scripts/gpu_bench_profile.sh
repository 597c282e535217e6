#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/bench_profile}
mkdir -p $OUT
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { cat $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash scripts/profile.sh $OUT/prof && python scripts/summarize_profile.py $OUT/prof $OUT/prof_summary.md "Round 1 (fast path) - step kernel, BASELINE config 2 (FrozenLake map1, 65,536 envs x 2 agents), MI355X" && cat $OUT/prof_summary.md
