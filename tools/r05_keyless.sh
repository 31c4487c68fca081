#!/bin/bash
# top-K insertion network A/B: parity tests that lean on the lists, then one-partition timing
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py tests/test_gpu_c1.py -x -q --timeout 300 --timeout-method thread > "$OUT/t.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/t.log"; exit 1; }
tail -1 "$OUT/t.log"
bash tools/r05_k2bknobs.sh "$OUT" klold
