mkdir -p gpurun_out/pol
for rep in 1 2; do
for lib in multiagent-rl-rm_amd/rmx/librmx.so multiagent-rl-rm_amd/csrc/build/librmx_exp_ldnt.so multiagent-rl-rm_amd/csrc/build/librmx_exp_stnt.so multiagent-rl-rm_amd/csrc/build/librmx_exp_both.so multiagent-rl-rm_amd/csrc/build/librmx_exp_stdef.so; do
  RMX_LIB=$lib timeout -k 10 200 python -u scripts/variants.py --configs 2,5 --variants fast:256 --n-envs 8388608 --steps 50 --rollout 0 > gpurun_out/pol/one.log 2>&1 || { cat gpurun_out/pol/one.log; exit 1; }
  grep config gpurun_out/pol/one.log | sed "s|^|$(basename $lib) big rep=$rep |" >> gpurun_out/pol/ab.log
  RMX_LIB=$lib timeout -k 10 200 python -u scripts/variants.py --configs 2,5 --variants fast:64 --steps 500 --rollout 0 > gpurun_out/pol/one.log 2>&1 || { cat gpurun_out/pol/one.log; exit 1; }
  grep config gpurun_out/pol/one.log | sed "s|^|$(basename $lib) small rep=$rep |" >> gpurun_out/pol/ab.log
done; done
