#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# K2b knob A/B on one C2 partition (tools/c2_part.py): variants under ab/, interleaved
set -uo pipefail
OUT=${1:?outdir}; shift; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do for v in default "$@"; do
  if [ "$v" = default ]; then unset HDBMI_LIB; else export HDBMI_LIB=$PWD/ab/$v/libhdbmi.so; fi
  echo -n "$v "; timeout -k 10 200 python -u tools/c2_part.py 5 2>>gpurun_out/tools_stderr.log | tail -1
done; done > "$OUT/ab.log" 2>&1
cat "$OUT/ab.log"
