# round 6, pass p: ALL5 (timing build: the five actions' M4 records fetched from the state, the action loaded last and
# only selecting) — its parity on the full-size / golden / queue GPU tests, then bench.py --config 2 / 3 / 4 (the
# bench's own fresh-action windows) with the shipping and the ALL5 library alternated
set -o pipefail
O=gpurun_out/r06p
mkdir -p $O
EX=$PWD/multiagent-rl-rm_amd/csrc/build/librmx_exp_all5.so
RMX_LIB=$EX timeout -k 10 700 python -u -m pytest tests/test_engine_gpu.py tests/test_queue_gpu.py tests/test_random_maps_gpu.py \
  -m gpu -q -x --timeout 300 --timeout-method thread -k "not library_is_the_hip_build" -p no:cacheprovider \
  > $O/tests_all5.txt 2>&1 && tail -1 $O/tests_all5.txt && \
QUICK="--steps 1000 --warmup 100 --no-cpu-baseline --no-rollout --large-envs 0 --dict-seconds 0 --rs-configs="
for rep in 1 2 3; do for lib in head all5; do for c in 2 3 4; do
  if [ $lib = all5 ]; then export RMX_LIB=$EX; else unset RMX_LIB; fi
  timeout -k 10 300 python -u bench.py --config $c $QUICK --detail $O/d_${lib}_c${c}_$rep.json > $O/b_${lib}_c${c}_$rep.json 2> $O/b.err || exit 1
  echo "$lib cfg=$c rep=$rep $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(round(d['ms_per_step']*1e3,4), round(d['us_per_step_event'],4), r.get('avg_launch_us_profile'), r.get('chain_launch_us'), d['parity']['rate'] if d.get('parity') else None)" $O/b_${lib}_c${c}_$rep.json)"
done; done; done
