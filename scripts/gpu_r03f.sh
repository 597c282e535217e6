#!/bin/bash
set -o pipefail
OUT=${OUT:-gpurun_out/r03f}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_sync_gpu.py tests/test_compat.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -40 $OUT/pytest.log; exit $rc; }
LIBS="multiagent-rl-rm_amd/rmx/librmx.so multiagent-rl-rm_amd/csrc/build/librmx_diag.so" OUT=$OUT/sync_ab bash scripts/gpu_sync_ab.sh
timeout -k 10 200 python -u -c "import json, bench; print(json.dumps(bench.dict_api_leg(0, 2.0)))" > $OUT/dict.json 2> $OUT/dict.err; rc=$?; cat $OUT/dict.json; exit $rc
