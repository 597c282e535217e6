#!/bin/bash
# Same-box A/B of the synchronous call across builds (scripts/sync_ab.py), plus the mailbox floors.
set -o pipefail
OUT=${OUT:-gpurun_out/sync_ab}
mkdir -p $OUT
timeout -k 10 90 ./scripts/sync_floor host > $OUT/floor.log 2>&1 || { cat $OUT/floor.log; exit 1; }
cat $OUT/floor.log
for rep in 1 2 3; do
  for lib in ${LIBS:-multiagent-rl-rm_amd/rmx/librmx.so}; do
    RMX_LIB=$lib timeout -k 10 120 python -u scripts/sync_ab.py >> $OUT/ab.log 2> $OUT/err.log || { cat $OUT/err.log; exit 1; }
  done
done
cat $OUT/ab.log
