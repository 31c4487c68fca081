#!/bin/bash
# K6 union-find accesses as agent-scope atomics instead of volatile: flat tests + per-partition time
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_ssort.py -x -q --timeout 300 --timeout-method thread -k "flat" > "$OUT/t_flat.log" 2>&1 || { echo "flat tests failed"; tail -40 "$OUT/t_flat.log"; exit 1; }
tail -1 "$OUT/t_flat.log"
for r in 1 2 3; do timeout -k 10 200 python -u tools/c2_part.py 5 2>>"$OUT/stderr.log" | tail -1; done > "$OUT/part.log" 2>&1
cat "$OUT/part.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o part --output-format csv -- python3 tools/c2_part.py 5 > /dev/null 2>&1 || echo "prof failed"
