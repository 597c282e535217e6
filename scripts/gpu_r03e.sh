#!/bin/bash
set -o pipefail
OUT=${OUT:-gpurun_out/r03e}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_random_maps_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "slip or golden or checkpoint" > $OUT/pytest.log 2>&1; rc=$?; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS="multiagent-rl-rm_amd/rmx/librmx.so multiagent-rl-rm_amd/csrc/build/librmx_exp_fenced.so multiagent-rl-rm_amd/csrc/build/librmx_diag.so" OUT=$OUT/sync_ab bash scripts/gpu_sync_ab.sh
