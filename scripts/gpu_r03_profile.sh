#!/bin/bash
# Round-3 evidence at HEAD: per-config copy floors (floor_bench cfg), kernel-trace + FETCH/WRITE passes of every
# BASELINE config, the 8.4M-env diagnostic and the slip steps (profile_configs.sh), one SQ-counter pass of config 3,
# and last (a host fault ends the call) floor_bench under the kernel tracer with the fault reporter.
set -o pipefail
OUT=${OUT:-gpurun_out/r03prof}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 120 ./scripts/floor_bench cfg > $OUT/floor_cfg.log 2>&1 || { cat $OUT/floor_cfg.log; exit 1; }
cat $OUT/floor_cfg.log
bash scripts/profile_configs.sh $OUT/prof || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d $OUT/sq3 -o sq -- python3 bench.py --config 3 \
  --graph 0 --steps 100 --warmup 10 --windows 1 --spin-ms 0 --no-cpu-baseline --no-rollout --large-envs 0 \
  --dict-seconds 0 > $OUT/sq3.json 2> $OUT/sq3.err || { tail -5 $OUT/sq3.err; exit 1; }
echo "sq3 done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/floorprof -o fp -- ./scripts/floor_bench \
  > $OUT/floor_prof.log 2>&1; echo "floor_bench under the tracer: exit $?"; tail -3 $OUT/floor_prof.log
