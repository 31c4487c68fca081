#!/bin/bash
# quick C4 screen A/B (no tests): variants under ab/
set -uo pipefail
OUT=$(readlink -f "${1:?outdir}"); shift
mkdir -p "$OUT"; export TMPDIR=/tmp
AB_REPS=${AB_REPS:-1} timeout -k 10 900 bash tools/ab_c4.sh "$@" > "$OUT/ab.log" 2>&1 || { echo "ab failed"; cat "$OUT/ab.log"; exit 1; }
cat "$OUT/ab.log"
