#!/bin/bash
# round 4 closing profiles: C2 (kernel stats + PMC passes) and C4 (stats + FETCH/WRITE).  Usage: bash tools/r04_prof.sh <outdir>
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 bash tools/profile_bench.sh "$OUT/prof_c2" > "$OUT/prof_c2.log" 2>&1 || { echo "c2 profile failed"; exit 1; }
timeout -k 10 560 bash tools/r04_c4prof.sh "$OUT/c4_final" > "$OUT/c4prof.log" 2>&1 || { echo "c4 profile failed"; exit 1; }
echo done
