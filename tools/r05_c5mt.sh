#!/bin/bash
# C5 vs local-model threads (HDB_MODEL_THREADS) at 8 / 12 hardware queues
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in "6 8" "8 12" "4 8"; do set -- $v
  HDB_MODEL_THREADS=$1 HDB_HW_QUEUES=$2 timeout -k 10 400 python -u bench.py --workload c5 --phases --no-cpu-baseline > "$OUT/c5_t$1_q$2.json.log" 2>"$OUT/c5_t$1_q$2.err" || { echo c5 failed; tail "$OUT/c5_t$1_q$2.err"; exit 1; }
  tail -1 "$OUT/c5_t$1_q$2.json.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 threads $1 q$2', round(d['ms_per_step'],1), (d.get('predicted_scaling') or {}).get('speedup'))"; done
