# round 6, pass k: the queue's dispatch timing (rmx_queue_timing) — its GPU tests; what dispatch profiling on the
# queue costs untimed windows (RMX_QUEUE_PROFILE=0 vs default, alternated); the default bench, whose roofline now
# carries this run's command-processor dispatch stamps (avg_launch_us_profile / frac_profile)
set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_queue_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread \
  -k "dispatch_timing or seq_equals_steps or longer_than" -p no:cacheprovider > $O/tests_timing.txt 2>&1 && \
tail -1 $O/tests_timing.txt && \
for rep in 1 2 3; do for pf in 1 0; do
  RMX_QUEUE_PROFILE=$pf timeout -k 10 200 python -u scripts/trace_window.py --config 2 > $O/tw_p${pf}_$rep.json 2> $O/tw.err \
    || exit 1; echo "profile=$pf rep=$rep $(cat $O/tw_p${pf}_$rep.json)"; done; done && \
timeout -k 10 600 python -u bench.py --detail $O/bench_detail_n1.json > $O/bench_n1.json 2> $O/bench_n1.err && \
python3 scripts/dispatch_times_summary.py $O/bench_detail_n1.json --md $O/dispatch_times.md > /dev/null && \
cat $O/dispatch_times.md && tail -c 1200 $O/bench_n1.json
