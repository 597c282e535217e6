# round 6, pass s: the final tree's rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of every BASELINE config
# (eager launches, scripts/gpu.sh profile), for profiles/ beside this round's bench lines
set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
for c in 2 3 4 5; do
  bash scripts/gpu.sh profile $O cfg$c --config $c --steps 100 --warmup 10 || exit 1
done
