#!/bin/bash
# Same-box A/B of the statistics report (scripts/stats_probe.py) over several library builds.
#   LIBS="a.so b.so" REPS=3 bash scripts/gpu_stats_ab.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/stats_ab}
mkdir -p "$OUT"
for rep in $(seq 1 ${REPS:-3}); do
  for lib in $LIBS; do
    RMX_LIB=$lib timeout -k 10 120 python -u scripts/stats_probe.py ${K:-20} >> "$OUT/ab.log" 2> "$OUT/err.log" || { cat "$OUT/err.log"; exit 1; }
    tail -1 "$OUT/ab.log"
  done
done
