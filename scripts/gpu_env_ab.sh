#!/bin/bash
# HIP runtime knobs vs the K = 20 window and the 500-step chain (scripts/report_probe.py), same box.
#   bash scripts/gpu_env_ab.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/envab}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # tag, env assignments...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python3 -u scripts/report_probe.py --reps 31 > "$OUT/$tag.k20.json" 2> "$OUT/$tag.err" || { tail -5 "$OUT/$tag.err"; return 1; }
  env "$@" timeout -k 10 120 python3 -u scripts/report_probe.py --steps 500 --reps 7 > "$OUT/$tag.k500.json" 2>> "$OUT/$tag.err" || { tail -5 "$OUT/$tag.err"; return 1; }
  echo "$tag k20 $(python3 -c "import json;d=json.load(open('$OUT/$tag.k20.json'));print(d['steps#1'],d['steps+fused#1'])") k500 $(python3 -c "import json;d=json.load(open('$OUT/$tag.k500.json'));print(d['steps#1'])")"
}
for round in 1 2; do
  run base$round A=1 || exit 1
  run devka1_$round HIP_FORCE_DEV_KERNARG=1 || exit 1
  run devka0_$round HIP_FORCE_DEV_KERNARG=0 || exit 1
  run pcap0_$round DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
  run batch1_$round DEBUG_HIP_GRAPH_BATCH_SIZE=1 || exit 1
  run batch64_$round DEBUG_HIP_GRAPH_BATCH_SIZE=64 || exit 1
done
# the dispatch headers (barrier / acquire / release fence scopes) of a few graph-replayed step launches
AMD_LOG_LEVEL=4 timeout -k 10 120 python3 -u scripts/report_probe.py --reps 1 > /dev/null 2> "$OUT/log4.err"
grep -m 12 "Dispatch Header" "$OUT/log4.err" > "$OUT/headers.txt"
cat "$OUT/headers.txt" | cut -c1-400
rm -f "$OUT/log4.err"
