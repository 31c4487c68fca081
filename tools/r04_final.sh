#!/bin/bash
# round 4 final check on the GPU box: full GPU test suite, smoke(), default bench (C2), C2 profile
# (kernel stats + PMC passes), C4 line + profile, C5 line with phases.  Usage: bash tools/r04_final.sh <outdir>
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gputest.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$OUT/gputest.log"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; exit 1; }
echo done
