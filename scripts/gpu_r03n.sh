#!/bin/bash
set -o pipefail
OUT=${OUT:-gpurun_out/r03n}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -q -rf -k "randstart" --timeout 100 --timeout-method thread \
  > $OUT/pytest.log 2>&1; rc=$?; grep -E "PASS|FAIL|passed|failed" $OUT/pytest.log | tail -40; exit 0
