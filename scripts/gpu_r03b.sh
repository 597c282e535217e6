set -o pipefail
OUT=${OUT:-gpurun_out/r03b}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_sync_gpu.py tests/test_compat.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -45 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import json, bench; print(json.dumps(bench.dict_api_leg(0, 2.0)))" > $OUT/dict.json 2> $OUT/dict.err; rc=$?; cat $OUT/dict.json; tail -5 $OUT/dict.err; exit $rc
