#!/bin/bash
# C5 whole job (phases, predicted scaling, K2b roofline), cooperative Prim slots 4 vs 6
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --workload c5 --phases > "$OUT/bench_c5.json.log" 2>&1 || { echo "c5 failed"; tail -20 "$OUT/bench_c5.json.log"; exit 1; }
HDB_PRIM_COOP_SLOTS=6 timeout -k 10 300 python -u bench.py --workload c5 --phases --no-cpu-baseline > "$OUT/bench_c5_spec.json.log" 2>&1 || { echo "c5 spec failed"; tail -20 "$OUT/bench_c5_spec.json.log"; exit 1; }
echo done
