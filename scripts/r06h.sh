# round 6, pass h: smoke, the new output-check GPU test, the default bench (driver form) at the final tree
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
bash scripts/gpu.sh smoke $O && \
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread \
  -k output_tensors -p no:cacheprovider > $O/tests_out.txt 2>&1 && tail -1 $O/tests_out.txt && \
timeout -k 10 600 python -u bench.py --detail $O/bench_detail_n1.json > $O/bench_n1.json 2> $O/bench_n1.err && \
cat $O/bench_n1.json
