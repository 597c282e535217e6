# round 6, pass f: VERDICT r05 item 7 — slip's reseed moved to the episode's last step (timing build lateseed) vs the
# shipping kernels: 500-step graphs with slip, libraries alternated; bench --slip chains; SQ counters of config 2
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"
HEAD=multiagent-rl-rm_amd/rmx/librmx.so
LS=multiagent-rl-rm_amd/csrc/build/librmx_exp_lateseed.so
REPS=4 bash scripts/gpu.sh libs $O ls "$HEAD $LS" --configs 2,3,4,5 --variants fast:64 --stochastic 1 && \
bash scripts/gpu.sh bench $O slip_head --slip --steps 500 --warmup 20 --no-cpu-baseline --large-envs 0 --dict-seconds 0 \
  --rs-configs= --detail $O/detail_slip_head.json && \
RMX_LIB=$PWD/$LS bash scripts/gpu.sh bench $O slip_ls --slip --steps 500 --warmup 20 --no-cpu-baseline --large-envs 0 \
  --dict-seconds 0 --rs-configs= --detail $O/detail_slip_ls.json && \
bash scripts/gpu.sh pmc $O sq_head "$SQ" --config 2 --slip --steps 100 --warmup 10 && \
RMX_LIB=$PWD/$LS bash scripts/gpu.sh pmc $O sq_ls "$SQ" --config 2 --slip --steps 100 --warmup 10
