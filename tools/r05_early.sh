#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# K2b early-round wave size A/B on one C2 partition (tools/c2_part.py), interleaved
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do for v in "0 5" "32 4" "32 2" "32 5" "16 3"; do set -- $v
  echo -n "early_pts=$1 rounds=$2 "; HDB_BOR_EARLY_PTS=$1 HDB_BOR_EARLY_ROUNDS=$2 timeout -k 10 200 python -u tools/c2_part.py 5 2>>gpurun_out/tools_stderr.log | tail -1
done; done > "$OUT/early.log" 2>&1
cat "$OUT/early.log"
