#!/bin/bash
# C5 at 12 and 16 hardware queues
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for q in 12 16; do HDB_HW_QUEUES=$q timeout -k 10 500 python -u bench.py --workload c5 --phases --no-cpu-baseline > "$OUT/c5_q$q.json.log" 2>"$OUT/c5_q$q.err" || { echo c5 failed; tail "$OUT/c5_q$q.err"; exit 1; }
  tail -1 "$OUT/c5_q$q.json.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 q$q', round(d['ms_per_step'],1), (d.get('predicted_scaling') or {}).get('speedup'))"; done
