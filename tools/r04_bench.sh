#!/bin/bash
# round 4 bench + profiles: C2 default line (with the CPU baseline), its rocprof stats + PMC
# passes, the C4 line + profile, the C5 line with phases.  Usage: bash tools/r04_bench.sh <outdir>
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > "$OUT/bench_c2.json.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench_c2.json.log"; exit 1; }
timeout -k 10 600 bash tools/profile_bench.sh "$OUT/prof_c2" > "$OUT/prof_c2.log" 2>&1 || { echo "profile failed"; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4 > "$OUT/bench_c4.json.log" 2>&1 || { echo "bench c4 failed"; exit 1; }
timeout -k 10 300 python -u bench.py --workload c5 --phases > "$OUT/bench_c5.json.log" 2>&1 || { echo "bench c5 failed"; exit 1; }
echo done
