#!/bin/bash
# quick check of the current build: tree tests + three one-partition runs
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py -x -q --timeout 300 --timeout-method thread > "$OUT/t_tree.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/t_tree.log"; exit 1; }
tail -1 "$OUT/t_tree.log"
for r in 1 2 3; do timeout -k 10 200 python -u tools/c2_part.py 5 2>>"$OUT/stderr.log" | tail -1; done > "$OUT/part.log" 2>&1
cat "$OUT/part.log"
