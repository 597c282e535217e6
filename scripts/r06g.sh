# round 6, pass g: FrozenLake slip with every outcome's record fetched before the reseed and the draws (timing build
# spec): its parity on the slip / stochastic GPU tests, then 500-step graphs with slip vs the shipping kernels, SQ counters
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"
HEAD=multiagent-rl-rm_amd/rmx/librmx.so
SP=multiagent-rl-rm_amd/csrc/build/librmx_exp_spec.so
RMX_LIB=$PWD/$SP timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
  -k "slip or stochastic or rng or randstart" -p no:cacheprovider > $O/tests_spec.txt 2>&1 && tail -2 $O/tests_spec.txt && \
REPS=4 bash scripts/gpu.sh libs $O sp "$HEAD $SP" --configs 2,3,4,5 --variants fast:64 --stochastic 1 && \
RMX_LIB=$PWD/$SP bash scripts/gpu.sh pmc $O sq_sp "$SQ" --config 2 --slip --steps 100 --warmup 10 && \
RMX_LIB=$PWD/$SP bash scripts/gpu.sh pmc $O sq_sp3 "$SQ" --config 3 --slip --steps 100 --warmup 10 && \
bash scripts/gpu.sh pmc $O sq_head3 "$SQ" --config 3 --slip --steps 100 --warmup 10
