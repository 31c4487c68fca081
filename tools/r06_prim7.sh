#!/bin/bash
# slots 7 (per-wave publish) vs slots 4: parity tests, then the 16k x 8 Prim / bubble Prim step cost
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "coop or prim or local_model or quicksort" > "$OUT/t_prim.log" 2>&1 || { echo "prim tests failed"; tail -30 "$OUT/t_prim.log"; exit 1; }
tail -2 "$OUT/t_prim.log"
for s in 4 7 4 7; do echo "slots=$s"; HDB_PRIM_COOP_SLOTS=$s timeout -k 10 120 python -u tools/prim_xcd_bench.py 16384 8 2>>"$OUT/stderr.log" | grep "xcd=1"; done > "$OUT/ab.log" 2>&1
cat "$OUT/ab.log"
for s in 4 7; do echo "slots=$s lm"; HDB_PRIM_COOP_SLOTS=$s timeout -k 10 120 python -u tools/lm_bench.py 16384 8 3 2>>"$OUT/stderr.log" | head -2; done >> "$OUT/ab.log" 2>&1
tail -6 "$OUT/ab.log"
