#!/bin/bash
# Same-box A/B of several builds of librmx.so, alternated REPS times (scripts/variants.py, default variant).
#   LIBS="a.so b.so" CFGS=2,5 REPS=3 bash scripts/gpu_libs_ab.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/libs_ab}
mkdir -p "$OUT"
for rep in $(seq 1 ${REPS:-3}); do
  for lib in $LIBS; do
    RMX_LIB=$lib timeout -k 10 200 python -u scripts/variants.py --configs ${CFGS:-2,5} --variants ${VARS:-fast:64} \
      --steps ${STEPS:-500} --rollout 0 > "$OUT/one.log" 2>&1 || { cat "$OUT/one.log"; exit 1; }
    grep config "$OUT/one.log" | sed "s|^|$(basename $lib) rep=$rep |"
  done
done | tee "$OUT/ab.log"
