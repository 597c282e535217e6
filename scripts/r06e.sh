# round 6, pass e: smoke, then the N > 1 path on one GPU (gloo rehearsal: ranks share the device) at 2 and 4 ranks
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
bash scripts/gpu.sh smoke $O && \
RMX_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --large-envs 0 \
  --dict-seconds 0 --detail $O/detail_gloo2.json > $O/bench_gloo2.json 2> $O/bench_gloo2.err && tail -c 400 $O/bench_gloo2.json && \
RMX_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 4 --steps 20 --warmup 5 --no-cpu-baseline --large-envs 0 \
  --dict-seconds 0 --rs-configs= --detail $O/detail_gloo4.json > $O/bench_gloo4.json 2> $O/bench_gloo4.err && tail -c 400 $O/bench_gloo4.json
