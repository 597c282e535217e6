#!/bin/bash
# One GPU pass at HEAD: smoke, the whole -m gpu suite, the bench in the driver's form (--steps 20 --warmup 5).
#   bash scripts/gpu_round.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -30 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=20 -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench20.json" 2> "$OUT/bench20.err" || { tail -30 "$OUT/bench20.err"; exit 1; }
cat "$OUT/bench20.json"
timeout -k 10 400 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -30 "$OUT/bench_default.err"; exit 1; }
cat "$OUT/bench_default.json"
