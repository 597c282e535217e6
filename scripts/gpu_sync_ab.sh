#!/bin/bash
# K=20 window cost by hipSetDeviceFlags scheduling mode (scripts/stats_probe.py), alternated
set -o pipefail
OUT=${1:-gpurun_out/sync}
mkdir -p "$OUT"
for rep in 1 2 3; do
  for fl in "" 1 2 4; do
    RMX_PROBE_DEVFLAGS=$fl timeout -k 10 120 python -u scripts/stats_probe.py 20 > "$OUT/one.log" 2> "$OUT/err.log" || { cat "$OUT/one.log" "$OUT/err.log"; exit 1; }
    tail -1 "$OUT/one.log" | tee -a "$OUT/ab.log"
  done
done
