#!/bin/bash
# random starts: draws of the next episode's shuffle per step (kRsDrawsPerStep) 0 / 8 / 16 / 32, same box
set -o pipefail
OUT=${OUT:-gpurun_out/r03v}
mkdir -p $OUT
for rep in 1 2; do for k in 0 8 16 32; do
  RMX_LIB=multiagent-rl-rm_amd/csrc/build/librmx_$( [ $k = 8 ] && echo rsk8 || echo exp_rsk$k ).so timeout -k 10 200 python -u scripts/variants.py \
    --random-starts 1 --configs 2,4 --variants fast:64 --rollout 0 > $OUT/one.log 2>&1 || { cat $OUT/one.log; exit 1; }
  grep config $OUT/one.log | sed "s|^|K=$k rep=$rep |"
done; done | tee $OUT/ab.log
