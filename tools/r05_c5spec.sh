#!/bin/bash
# C5 with 8 hardware queues: cooperative Prim slots 4 (default) vs 6 (speculative)
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in 6 4; do HDB_PRIM_COOP_SLOTS=$v timeout -k 10 400 python -u bench.py --workload c5 --phases --no-cpu-baseline > "$OUT/c5_s$v.json.log" 2>"$OUT/c5_s$v.err" || { echo c5 failed; tail "$OUT/c5_s$v.err"; exit 1; }
  tail -1 "$OUT/c5_s$v.json.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('slots $v', round(d['ms_per_step'],1), (d.get('predicted_scaling') or {}).get('speedup'), r.get('us_per_step'))"; done
