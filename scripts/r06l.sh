# round 6, pass l: dispatch timing with GPU-only (interrupt-free) timing signals; the window's completion signal with
# and without its interrupt (RMX_QUEUE_DONE=gpu), K = 20 and 500, alternated; the timing GPU tests; a bench
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_queue_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread \
  -k "dispatch_timing or seq_equals_steps or longer_than or falls_back" -p no:cacheprovider > $O/tests_timing.txt 2>&1 && \
tail -1 $O/tests_timing.txt && \
for rep in 1 2 3; do for dn in irq gpu; do for k in 20 500; do
  RMX_QUEUE_DONE=$dn timeout -k 10 200 python -u scripts/trace_window.py --config 2 --k $k --windows 40 \
    > $O/tw_${dn}_k${k}_$rep.json 2> $O/tw.err || exit 1
  echo "done=$dn k=$k rep=$rep $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['us_per_step_wall_median'],4), round(d['us_per_step_wall_min'],4))" $O/tw_${dn}_k${k}_$rep.json)"
done; done; done && \
timeout -k 10 600 python -u bench.py --detail $O/bench_detail_n1.json > $O/bench_n1.json 2> $O/bench_n1.err && \
python3 scripts/dispatch_times_summary.py $O/bench_detail_n1.json --md $O/dispatch_times.md > /dev/null && \
cat $O/dispatch_times.md && tail -c 300 $O/bench_n1.json
