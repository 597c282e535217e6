# round 6, pass d: the step kernel's dispatch span at the bench's cadence (diag build, entry / exit stamps on a
# back-to-back graph) and a counter pass with the kernel trace (GRBM / SQ busy cycles per dispatch), configs 2-5
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
DIAG=$PWD/multiagent-rl-rm_amd/csrc/build/librmx_diag.so
PROF_BENCH="--graph 0 --dispatch graph --spin-ms 50 --no-cpu-baseline --no-rollout --large-envs 0 --dict-seconds 0 --rs-configs= --windows 1 --chain 0"
for c in 2 3 4 5; do
  RMX_LIB=$DIAG timeout -k 10 120 python3 scripts/stamps.py --config $c --steps 200 --edges 1 --samples 30 \
    > $O/stamps_edges_$c.json 2> $O/stamps_$c.err || { tail -20 $O/stamps_$c.err; exit 1; }
  cat $O/stamps_edges_$c.json
done
RMX_LIB=$DIAG timeout -k 10 120 python3 scripts/stamps.py --config 2 --steps 200 --samples 5 > $O/stamps_full_2.json \
  2> $O/stamps_full.err || { tail -20 $O/stamps_full.err; exit 1; }
for c in 2 3 4 5; do
  d=$O/ctr$c; mkdir -p $d
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVES \
    --output-format csv -d $d/pmc -o pmc -- python3 bench.py $PROF_BENCH --config $c --steps 100 --warmup 10 \
    > $d/bench.json 2> $d/pmc.err || { tail -20 $d/pmc.err; exit 1; }
  echo "ctr $c done"
done
timeout -k 10 600 python3 bench.py --detail $O/detail_n1.json > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
echo bench done
