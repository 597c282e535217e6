#!/bin/bash
# Config 3 and slip characterisation (round 3): live per-step times of table modes / block sizes for config 3, the
# lookup ablations (diag build), in-kernel stamps of configs 2 and 3, slip on the fast kernel vs the generic one
# (configs 2 and 3 with their env's slip switch); last, floor_bench under the kernel tracer with its graphs kept
# alive until exit (the round-2 / round-3 SIGSEGV came right after graphs of the previous size were destroyed).
set -o pipefail
OUT=${OUT:-gpurun_out/r03h}
export TMPDIR=/tmp
mkdir -p $OUT
DIAG=multiagent-rl-rm_amd/csrc/build/librmx_diag.so
timeout -k 10 300 python -u scripts/variants.py --configs 3 --variants fast:64,fastX:64,fastM:64,fastG:64,fast:128,fast:256,fast:64 --rollout 0 > $OUT/cfg3_variants.log 2>&1 || { tail -20 $OUT/cfg3_variants.log; exit 1; }
cat $OUT/cfg3_variants.log
RMX_LIB=$DIAG timeout -k 10 300 python -u scripts/variants.py --configs 3,2 --variants fast:64,fast:64:4096,fast:64:8192,fast:64:1,fast:64 --rollout 0 > $OUT/ablate.log 2>&1 || { tail -20 $OUT/ablate.log; exit 1; }
cat $OUT/ablate.log
for c in 3 2; do
  timeout -k 10 200 python -u scripts/stamps.py --config $c > $OUT/stamps_cfg$c.log 2>&1 || { tail -20 $OUT/stamps_cfg$c.log; exit 1; }
  cat $OUT/stamps_cfg$c.log
done
timeout -k 10 300 python -u scripts/variants.py --stochastic 1 --configs 2,3 --variants fast:64,tpe:256,fast:64,tpe:256 --rollout 1 > $OUT/slip_variants.log 2>&1 || { tail -20 $OUT/slip_variants.log; exit 1; }
cat $OUT/slip_variants.log
FLOOR_KEEP_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/floorprof -o fp -- ./scripts/floor_bench > $OUT/floor_prof_keep.log 2>&1; echo "floor_bench (graphs kept) under the tracer: exit $?"; grep -c n_envs $OUT/floor_prof_keep.log
