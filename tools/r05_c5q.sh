#!/bin/bash
# C2 default line (bench.py now sets 8 hardware queues) and C5 at 4 vs 8 queues
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 40 --no-cpu-baseline > "$OUT/c2.json.log" 2>"$OUT/c2.err" || { echo c2 failed; tail "$OUT/c2.err"; exit 1; }
tail -1 "$OUT/c2.json.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', round(d['ms_per_step'],3), round(d['value']/1e6,1), d['config']['hw_queues'], d['schema'])"
for q in 4 8; do HDB_HW_QUEUES=$q timeout -k 10 500 python -u bench.py --workload c5 --phases --no-cpu-baseline > "$OUT/c5_q$q.json.log" 2>"$OUT/c5_q$q.err" || { echo c5 failed; tail "$OUT/c5_q$q.err"; exit 1; }
  tail -1 "$OUT/c5_q$q.json.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 q$q', round(d['ms_per_step'],1), (d.get('predicted_scaling') or {}).get('speedup'))"; done
