#!/bin/bash
# full GPU test suite + smoke
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gputest.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$OUT/gputest.log"; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail "$OUT/smoke.log"; exit 1; }
tail -3 "$OUT/gputest.log"; tail -2 "$OUT/smoke.log"
