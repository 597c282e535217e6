set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"
HEAD=multiagent-rl-rm_amd/rmx/librmx.so
T0=multiagent-rl-rm_amd/csrc/build/librmx_exp_t0.so
REPS=4 bash scripts/gpu.sh libs $O t0 "$HEAD $T0" --configs 4,2 --variants fast:64 && \
bash scripts/gpu.sh pmc $O sq_head "$SQ" --config 4 --steps 100 --warmup 10 && \
RMX_LIB=$PWD/$T0 bash scripts/gpu.sh pmc $O sq_t0 "$SQ" --config 4 --steps 100 --warmup 10 && \
bash scripts/gpu.sh twtrace $O tw2 2 && bash scripts/gpu.sh twtrace $O tw3 3 && \
bash scripts/gpu.sh twtrace $O tw4 4 && bash scripts/gpu.sh twtrace $O tw5 5 && \
bash scripts/gpu.sh bench $O k20 --steps 20 --warmup 5 --detail $O/detail_k20.json
