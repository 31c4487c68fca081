#!/bin/bash
# C2 line + its rocprof kernel stats (round 5)
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > "$OUT/bench_c2.json.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench_c2.json.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/prof_bench.json.log" 2> "$OUT/stats.err" || { echo "prof failed"; exit 1; }
echo done
