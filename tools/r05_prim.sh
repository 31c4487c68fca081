#!/bin/bash
# speculative cooperative Prim: parity tests, then slots 4 vs 6 step cost
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "prim_coop or cooperative" --timeout 300 --timeout-method thread > "$OUT/t_prim.log" 2>&1 || { echo "prim tests failed"; tail -40 "$OUT/t_prim.log"; exit 1; }
for s in 4 6; do HDB_PRIM_COOP_SLOTS=$s timeout -k 10 200 python -u tools/prim_xcd_bench.py 16384 8 > "$OUT/bench_s$s.log" 2>&1 || { echo "bench $s failed"; tail -5 "$OUT/bench_s$s.log"; exit 1; }; done
for s in 4 6; do HDB_PRIM_COOP_SLOTS=$s timeout -k 10 200 python -u tools/prim_xcd_bench.py 4096 16 > "$OUT/bench16_s$s.log" 2>&1 || { echo "bench16 $s failed"; exit 1; }; done
echo done
