#!/bin/bash
# bench.py --sync auto vs spin in the driver's form, alternated on one box (config 2 value and windows)
set -o pipefail
OUT=${1:-gpurun_out/syncspin}
mkdir -p "$OUT"
for rep in 1 2 3; do
  for mode in auto spin; do
    timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rollout --large-envs 0 \
      --sync $mode > "$OUT/$mode$rep.json" 2> "$OUT/$mode$rep.err" || { tail -5 "$OUT/$mode$rep.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$mode$rep.json')); print('$mode', $rep, round(d['value']/1e9,2), round(d['ms_per_step']*1e3,3), round(d['us_per_step_event'],3), [round(w['us_per_step_wall'],2) for w in d['windows']], {k: round(v['value']/1e9,1) for k, v in d['configs'].items()})"
  done
done
