#!/bin/bash
# FrozenLake random starts on the fast path: the random-start / slip / golden GPU tests, then the per-step timing
# (fast vs generic, step and rollout) beside the deterministic kernel.
set -o pipefail
OUT=${OUT:-gpurun_out/r03l}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_sync_gpu.py tests/test_compat.py -m gpu -x -q \
  -k "randstart or slip or stochastic or golden or checkpoint or save_load" --timeout 100 --timeout-method thread \
  > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -60 $OUT/pytest.log; exit $rc; }
timeout -k 10 300 python -u scripts/variants.py --random-starts 1 --configs 2,4 --variants fast:64,tpe:64 --rollout 1 > $OUT/randstart.log 2>&1 || { tail -20 $OUT/randstart.log; exit 1; }
cat $OUT/randstart.log
timeout -k 10 300 python -u scripts/variants.py --random-starts 1 --stochastic 1 --configs 2 --variants fast:64,tpe:64 --rollout 1 > $OUT/randstart_slip.log 2>&1 || { tail -20 $OUT/randstart_slip.log; exit 1; }
cat $OUT/randstart_slip.log
