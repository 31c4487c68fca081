#!/bin/bash
# C4 line profile: kernel-trace stats of the C4 bench, then its FETCH/WRITE passes (tools/profile_c4.sh).
# Usage: bash tools/r04_c4prof.sh <outdir>
set -uo pipefail
OUT=$(readlink -f "${1:?outdir}")
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o c4 --output-format csv -- \
    python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c4_stats.json.log" 2> "$OUT/stats.err" || { echo "stats pass failed"; exit 1; }
timeout -k 10 500 bash tools/profile_c4.sh "$OUT" > "$OUT/pmc.log" 2>&1 || { echo "pmc passes failed"; exit 1; }
echo done
