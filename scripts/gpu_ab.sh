#!/bin/bash
# A/B timing of step-kernel variants on the GPU box (scripts/variants.py), optionally with the diagnostic
# build.  Usage: bash scripts/gpu_ab.sh OUTDIR CONFIGS VARIANTS [diag]
#   e.g. bash scripts/gpu_ab.sh gpurun_out/ab 2,5 fast:256,fastlpe:256,tpe:256
#        bash scripts/gpu_ab.sh gpurun_out/ab 2 fast:256:0,fast:256:1 diag
set -o pipefail
OUT=$1; CFGS=$2; VARS=$3
mkdir -p "$OUT"
if [ "$4" = "diag" ]; then export RMX_LIB=multiagent-rl-rm_amd/csrc/build/librmx_diag.so; fi
timeout -k 10 300 python -u scripts/variants.py --configs "$CFGS" --variants "$VARS" --rollout 0 > "$OUT/ab.log" 2>&1
rc=$?; cat "$OUT/ab.log"; exit $rc
