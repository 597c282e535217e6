#!/bin/bash
# Same-box A/B of two builds of librmx.so (alternated twice): build/librmx_prev.so vs the in-tree one.
set -o pipefail
OUT=${OUT:-gpurun_out/lib_ab}
mkdir -p $OUT
for rep in 1 2; do
  for lib in multiagent-rl-rm_amd/csrc/build/librmx_prev.so multiagent-rl-rm_amd/rmx/librmx.so; do
    echo "# lib=$lib rep=$rep"
    RMX_LIB=$lib timeout -k 10 200 python -u scripts/variants.py --configs ${CFGS:-2,5} --variants ${VARS:-fast:256} --rollout 0 2>&1 | grep config || exit 1
  done
done | tee $OUT/ab.log
