#!/bin/bash
# closing C2 profile (kernel stats + PMC passes) of the final build.  Usage: bash tools/r04_prof2.sh <outdir>
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 bash tools/profile_bench.sh "$OUT/prof_c2" > "$OUT/prof_c2.log" 2>&1 || { echo "c2 profile failed"; exit 1; }
echo done
