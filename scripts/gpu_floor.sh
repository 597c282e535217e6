#!/bin/bash
# Launch-chain floors (scripts/floor_bench) next to the step kernels, in ONE call so that the numbers
# come from the same device and clock (MI355X devices differ by up to ~20% on this launch-bound shape).
set -o pipefail
OUT=${OUT:-gpurun_out/floor}
mkdir -p $OUT
timeout -k 10 60 ./scripts/floor_bench > $OUT/floor.log 2>&1; rc=$?; cat $OUT/floor.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/variants.py --configs ${CFGS:-2,3,4,5} --variants ${VARS:-fast:256,fastlpe:256,tpe:256} --rollout 0 > $OUT/var.log 2>&1; rc=$?; cat $OUT/var.log; exit $rc
