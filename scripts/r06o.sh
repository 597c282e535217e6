# round 6, pass o: the doorbell rung while a window's packets are written (after the first, then every 16) vs once at
# the end (RMX_QUEUE_EARLY=0): config 2 windows at K = 20 and 500 and config 3 at K = 20, alternated; then the queue
# tests (the window mechanics changed) and the smoke
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
for rep in 1 2 3; do for ea in 1 0; do for ck in "2 20" "2 500" "3 20"; do
  set -- $ck
  RMX_QUEUE_EARLY=$ea timeout -k 10 200 python -u scripts/trace_window.py --config $1 --k $2 --windows 40 \
    > $O/tw_e${ea}_c$1_k$2_$rep.json 2> $O/tw.err || exit 1
  echo "early=$ea cfg=$1 k=$2 rep=$rep $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['us_per_step_wall_median'],4), round(d['us_per_step_wall_min'],4), d['dispatch'])" $O/tw_e${ea}_c$1_k$2_$rep.json)"
done; done; done && \
timeout -k 10 900 python -u -m pytest tests/test_queue_gpu.py tests/test_raw_capi_gpu.py -m gpu -q -x --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/tests_queue.txt 2>&1 && tail -1 $O/tests_queue.txt && \
bash scripts/gpu.sh smoke $O
