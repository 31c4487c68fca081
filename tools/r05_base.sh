#!/bin/bash
# round 5 baseline on the box: one C2 partition at a time (wall + library timers), then the same
# under rocprofv3 kernel stats (each kernel alone).  Usage: bash tools/r05_base.sh <outdir>
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 200 python -u tools/c2_part.py 5 > "$OUT/c2_part.log" 2>&1 || { echo "c2_part failed"; tail -20 "$OUT/c2_part.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o part --output-format csv -- python3 tools/c2_part.py 4 > "$OUT/c2_prof.log" 2>&1 || { echo "prof failed"; tail -20 "$OUT/c2_prof.log"; exit 1; }
echo done
