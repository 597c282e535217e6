#!/bin/bash
# One GPU-box pass: parity suite, smoke, bench (N=1), concurrency + floor diagnostics, kernel-trace profile.
set -o pipefail
OUT=gpurun_out/${TAG:-check}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { cat "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ -n "$EXTRA" ]; then
  timeout -k 10 400 bash -c "$EXTRA" > "$OUT/extra.log" 2>&1 || { tail -30 "$OUT/extra.log"; exit 1; }
  tail -40 "$OUT/extra.log"
fi
