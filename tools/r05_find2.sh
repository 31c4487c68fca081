#!/bin/bash
# K6 interleaved finds: flat-label tests, then one-partition A/B (ab/flold = previous flat.hip)
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_c1.py tests/test_gpu_ssort.py -x -q --timeout 300 --timeout-method thread > "$OUT/t.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/t.log"; exit 1; }
tail -1 "$OUT/t.log"
bash tools/r05_k2bknobs.sh "$OUT" flold
