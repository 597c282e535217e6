set -o pipefail
mkdir -p gpurun_out/c43
for rep in 1 2; do
  for lib in multiagent-rl-rm_amd/csrc/build/librmx_prev.so multiagent-rl-rm_amd/rmx/librmx.so; do
    echo "# lib=$lib rep=$rep"
    RMX_FAST_STATS=wave RMX_LIB=$lib timeout -k 10 200 python -u scripts/variants.py --configs 2,5 --variants fast:256 --n-envs 8388608 --steps 20 --reps 3 --rollout 0 2>&1 | grep config || exit 1
  done
done > gpurun_out/c43/ab.log
