#!/bin/bash
# C5 kernel-trace stats (one whole-job run).  Usage: bash tools/r04_c5prof.sh <outdir>
set -uo pipefail
OUT=$(readlink -f "${1:?outdir}")
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o c5 --output-format csv -- \
    python3 bench.py --workload c5 --no-cpu-baseline > "$OUT/bench_c5_stats.json.log" 2> "$OUT/stats.err" || { echo "c5 stats failed"; exit 1; }
rm -f "$OUT"/stats/*kernel_trace.csv
echo done
