#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# K6 deep-depth kernel variants, one partition at a time (c2_part flat_labels timer)
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do
for cfg in "64 3 1" "2 0 0" "4 0 0" "6 0 0" "4 2 0" "4 1 0" "4 0 1" "4 3 0"; do
  set -- $cfg
  echo -n "deep=$1 root=$2 link=$3 "; HDB_FLAT_DEEP=$1 HDB_FLAT_DEEP_ROOT=$2 HDB_FLAT_DEEP_LINK=$3 timeout -k 10 100 python -u tools/c2_part.py 5 2>>gpurun_out/tools_stderr.log | tail -1 | sed 's/.*flat_labels/flat_labels/'
done; done > "$OUT/ab.log" 2>&1
echo done
