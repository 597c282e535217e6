#!/bin/bash
# bench.py --steps 20 --warmup 5 with and without NUMA pinning of the launching thread, alternated
set -o pipefail
OUT=${1:-gpurun_out/pin}
mkdir -p "$OUT"
for rep in 1 2 3; do
  for pin in none numa; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rollout --large-envs 0 --pin $pin \
      > "$OUT/b.json" 2> "$OUT/b.err" || { tail -20 "$OUT/b.err"; exit 1; }
    python - "$OUT/b.json" $pin $rep <<'PY' | tee -a "$OUT/ab.log"
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], d["config"].get("host_pin"), round(d["ms_per_step"] * 1e3, 3),
      [round(w["us_per_step_wall"], 2) for w in d["windows"]],
      {c: round(v["ms_per_step"] * 1e3, 3) for c, v in d["configs"].items()})
PY
  done
done
