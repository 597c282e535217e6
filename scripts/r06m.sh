# round 6, pass m: dispatch timing with a stamp stride (packets 0, m, 2m, ... and the last): the GPU tests, then the
# default bench, whose roofline carries the CP-clock dispatch time of its own queue windows
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_queue_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread \
  -k "dispatch_timing or seq_equals_steps or longer_than" -p no:cacheprovider > $O/tests_timing.txt 2>&1 && \
tail -1 $O/tests_timing.txt && \
timeout -k 10 600 python -u bench.py --detail $O/bench_detail_n1.json > $O/bench_n1.json 2> $O/bench_n1.err && \
python3 scripts/dispatch_times_summary.py $O/bench_detail_n1.json --md $O/dispatch_times.md > /dev/null && \
cat $O/dispatch_times.md && tail -c 300 $O/bench_n1.json
