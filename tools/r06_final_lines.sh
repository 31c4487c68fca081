#!/bin/bash
# round 6 closing lines (call 2 of 2, after tools/r06_final_prof.sh and its summaries copied into
# profiles/r06/): C2 default line with its CPU baseline, C4 line, C5 line with phases (the rank
# emulation of predicted_scaling) and its CPU baseline.  Usage: bash tools/r06_final_lines.sh <outdir>
set -uo pipefail
mkdir -p "${1:?outdir}"; OUT=$(readlink -f "$1"); export TMPDIR=/tmp
export HDB_NATIVE_BACKTRACE=1
timeout -k 10 400 python -u bench.py > "$OUT/bench_c2.json.log" 2> "$OUT/bench_c2.err" || { echo "c2 failed"; tail "$OUT/bench_c2.err"; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4 > "$OUT/bench_c4.json.log" 2> "$OUT/bench_c4.err" || { echo "c4 failed"; tail "$OUT/bench_c4.err"; exit 1; }
timeout -k 10 900 python -u bench.py --workload c5 --phases > "$OUT/bench_c5.json.log" 2> "$OUT/bench_c5.err" || { echo "c5 failed"; tail "$OUT/bench_c5.err"; exit 1; }
for f in bench_c2 bench_c4 bench_c5; do tail -1 "$OUT/$f.json.log" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}
print('$f', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],2), 'ms', 'lat', d.get('latency_ms_per_step'), 'roof', r.get('kernel'), r.get('frac'), 'traffic', r.get('traffic'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"; done
