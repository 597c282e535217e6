#!/bin/bash
# random starts ablations (timing only; ablated builds compute wrong positions by design), then the dict-API
# mailbox floor with the request word in host memory and in fine-grained device memory
set -o pipefail
OUT=${OUT:-gpurun_out/r03x}
mkdir -p $OUT
for rep in 1 2; do for x in HEAD NOCOOP NOUNDO NODRAWS NOSEED NOCELLS; do
  RMX_LIB=multiagent-rl-rm_amd/csrc/build/librmx_exp_$x.so timeout -k 10 200 python -u scripts/variants.py \
    --random-starts 1 --configs 2 --variants fast:64 --rollout 0 > $OUT/one.log 2>&1 || { cat $OUT/one.log; exit 1; }
  grep config $OUT/one.log | sed "s|^|$x rep=$rep |"
done; done | tee $OUT/ab.log
timeout -k 10 120 ./scripts/sync_floor > $OUT/sync_host.log 2>&1; echo "sync_floor host: exit $?"; cat $OUT/sync_host.log
timeout -k 10 120 ./scripts/sync_floor vram > $OUT/sync_vram.log 2>&1; echo "sync_floor vram: exit $?"; cat $OUT/sync_vram.log
