#!/bin/bash
# HEAD rocprofv3 evidence: kernel-trace + FETCH/WRITE per config (profile_configs.sh), one SQ pass of config 3
set -o pipefail
OUT=${OUT:-gpurun_out/r03z}
export TMPDIR=/tmp
mkdir -p $OUT
CFGS="2 3 4 5 hbm" bash scripts/profile_configs.sh $OUT/prof || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d $OUT/sq3 -o sq -- python3 bench.py --config 3 \
  --graph 0 --steps 100 --warmup 10 --windows 1 --spin-ms 0 --no-cpu-baseline --no-rollout --large-envs 0 \
  --dict-seconds 0 --chain 0 > $OUT/sq3.json 2> $OUT/sq3.err || { tail -5 $OUT/sq3.err; exit 1; }
echo "sq3 done"
