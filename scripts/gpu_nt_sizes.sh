#!/bin/bash
# kSkipRare (sc1 stores) vs kSkipRareNT (nt|sc1 stores) across env counts (variants.py, fast kernel, 256-thread WGs)
set -o pipefail
OUT=${1:-gpurun_out/nt}
mkdir -p "$OUT"
for rep in 1 2; do
  for n in 262144 1048576 2097152 8388608; do
    steps=$(( n >= 2097152 ? 50 : 200 ))
    timeout -k 10 240 python -u scripts/variants.py --configs 2,3,4,5 --variants fastR:256,fastT:256 --n-envs $n \
      --steps $steps --rollout 0 > "$OUT/one.log" 2>&1 || { cat "$OUT/one.log"; exit 1; }
    grep config "$OUT/one.log" | sed "s|^|n=$n rep=$rep |" >> "$OUT/ab.log"
  done
done
