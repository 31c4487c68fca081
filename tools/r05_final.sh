#!/bin/bash
# round 5 closing lines on the GPU box: C2 (default line with its CPU baseline) + rocprof stats +
# PMC passes, C4 line + stats + PMC, C5 line with phases and its CPU baseline.
# Usage (repo root, on the box): bash tools/r05_final.sh <outdir>
set -uo pipefail
OUT=$(readlink -f "${1:?outdir}")
mkdir -p "$OUT"; export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8  # as bench.py sets it (the profiler initialises HIP before bench.py runs)
timeout -k 10 400 python -u bench.py > "$OUT/bench_c2.json.log" 2> "$OUT/bench_c2.err" || { echo "c2 failed"; tail "$OUT/bench_c2.err"; exit 1; }
timeout -k 10 700 bash tools/profile_bench.sh "$OUT/prof_c2" > "$OUT/prof_c2.log" 2>&1 || { echo "c2 profile failed"; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4 > "$OUT/bench_c4.json.log" 2> "$OUT/bench_c4.err" || { echo "c4 failed"; tail "$OUT/bench_c4.err"; exit 1; }
timeout -k 10 600 bash tools/c4prof.sh "$OUT/c4_prof" > "$OUT/c4_prof.log" 2>&1 || { echo "c4 profile failed"; exit 1; }
timeout -k 10 600 python -u bench.py --workload c5 --phases > "$OUT/bench_c5.json.log" 2> "$OUT/bench_c5.err" || { echo "c5 failed"; tail "$OUT/bench_c5.err"; exit 1; }
for f in bench_c2 bench_c4 bench_c5; do tail -1 "$OUT/$f.json.log" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}
print('$f', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],2), 'ms', 'lat', d.get('latency_ms_per_step'), 'roof', r.get('kernel'), r.get('frac'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"; done
