#!/bin/bash
# Round-3 pass: the standard round (smoke, -m gpu suite, bench K=20 and default) at the working tree, then a
# same-box A/B of the HEAD library against the tree's (discount load issued after the table lookups).
set -o pipefail
OUT=${OUT:-gpurun_out/r03j}
mkdir -p $OUT
bash scripts/gpu_round.sh $OUT/round || exit 1
LIBS="multiagent-rl-rm_amd/csrc/build/librmx_head.so multiagent-rl-rm_amd/rmx/librmx.so" CFGS=3,5,2 REPS=3 \
  bash scripts/gpu_libs_ab.sh $OUT/ab
