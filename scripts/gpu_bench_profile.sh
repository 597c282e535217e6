#!/bin/bash
# Round-end style GPU pass: smoke, the default bench line, rocprof of the headline size and of the
# HBM-resident size (bandwidth regime), each summarised for profiles/.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/bench_profile}
TAG=${TAG:-r01}
mkdir -p $OUT
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { cat $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash scripts/profile.sh $OUT/prof && python scripts/summarize_profile.py $OUT/prof $OUT/prof_summary.md "$TAG - step kernel, BASELINE config 2 (FrozenLake map1, 65,536 envs x 2 agents), MI355X" || exit 1
bash scripts/profile.sh $OUT/prof_hbm "--no-cpu-baseline --no-rollout --large-envs 0 --n-envs 8388608 --steps 50 --warmup 5" && python scripts/summarize_profile.py $OUT/prof_hbm $OUT/prof_hbm_summary.md "$TAG - step kernel at an HBM-resident size (config 2 shape, 8,388,608 envs x 2 agents), MI355X" || exit 1
grep -h "step_fast\|step_kernel" $OUT/prof_summary.md $OUT/prof_hbm_summary.md
