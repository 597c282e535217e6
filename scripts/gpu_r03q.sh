#!/bin/bash
# floor_bench under rocprofv3 --kernel-trace with eager launch chains (FLOOR_EAGER=1): the clean tracer pass
set -o pipefail
OUT=${OUT:-gpurun_out/r03q}
mkdir -p $OUT
export TMPDIR=/tmp
FLOOR_EAGER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/floorprof -o fp -- ./scripts/floor_bench \
  > $OUT/floor_prof_eager.log 2>&1; rc=$?; echo "floor_bench eager under the tracer: exit $rc"; grep n_envs $OUT/floor_prof_eager.log | head -8
find $OUT/floorprof -name "*kernel_stats.csv" | head -3
exit $rc
