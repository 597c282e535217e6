# round 6, pass v: the N = 8 path on one GPU (gloo rehearsal: 8 ranks share the device) — the compact line at 8 ranks
set -o pipefail
O=gpurun_out/r06v
mkdir -p $O
RMX_BENCH_BACKEND=gloo timeout -k 10 900 python3 bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline --large-envs 0 \
  --dict-seconds 0 --rs-configs= --detail $O/detail_gloo8.json > $O/bench_gloo8.json 2> $O/bench_gloo8.err && \
wc -c $O/bench_gloo8.json && tail -c 600 $O/bench_gloo8.json
