set -o pipefail
for rep in 1 2; do for lib in multiagent-rl-rm_amd/csrc/build/librmx_prev.so multiagent-rl-rm_amd/rmx/librmx.so; do
RMX_LIB=$lib timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-rollout --large-envs 0 > gpurun_out/bab/b.json 2>/dev/null || exit 1
python3 -c "import json,sys; d=json.load(open('gpurun_out/bab/b.json')); print(sys.argv[1][-20:], round(d['value']/1e9,2), round(d['roofline']['avg_launch_us'],3), round(d['config4']['value']/1e9,1))" $lib
done; done
