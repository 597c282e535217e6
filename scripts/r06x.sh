# round 6, pass x: the exact final tree as the driver will run it — pytest -m gpu, smoke, bench.py (defaults)
set -o pipefail
O=gpurun_out/r06x
mkdir -p $O
bash scripts/gpu.sh tests $O final && bash scripts/gpu.sh smoke $O && \
timeout -k 10 600 python -u bench.py --detail $O/bench_detail_n1.json > $O/bench_n1.json 2> $O/bench_n1.err && \
tail -c 700 $O/bench_n1.json
