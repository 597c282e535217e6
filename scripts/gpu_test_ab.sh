#!/bin/bash
# GPU parity suite, then an A/B timing sweep (scripts/variants.py) on the same box.
set -o pipefail
OUT=${OUT:-gpurun_out/test_ab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/variants.py --configs ${CFGS:-2,3,4,5} --variants ${VARS:-fast:256,fastlpe:256,tpe:256} --rollout 0 > $OUT/var.log 2>&1; rc=$?; cat $OUT/var.log; exit $rc
