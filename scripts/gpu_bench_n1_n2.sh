set -o pipefail
mkdir -p gpurun_out/c53
timeout -k 10 300 python -u bench.py > gpurun_out/c53/n1.json 2> gpurun_out/c53/n1.err || exit 1
RMX_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/c53/n2.json 2> gpurun_out/c53/n2.err || exit 1
