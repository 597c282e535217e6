#!/bin/bash
# random starts: the GPU tests of the tree (first-occurrence undo, rollout on rs_step), then a same-box A/B of the
# previous commit's library (full undo over the row) against the tree's, step and rollout
set -o pipefail
OUT=${OUT:-gpurun_out/r03ab}
mkdir -p $OUT
bash scripts/gpu_r03n.sh || exit 1
for rep in 1 2 3; do for x in multiagent-rl-rm_amd/csrc/build/librmx_exp_prev.so multiagent-rl-rm_amd/rmx/librmx.so; do
  RMX_LIB=$x timeout -k 10 200 python -u scripts/variants.py \
    --random-starts 1 --configs 2,4 --variants fast:64 --rollout 1 > $OUT/one.log 2>&1 || { cat $OUT/one.log; exit 1; }
  grep config $OUT/one.log | sed "s|^|$(basename $x) rep=$rep |"
done; done | tee $OUT/ab.log
