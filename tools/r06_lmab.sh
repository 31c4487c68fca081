#!/bin/bash
# one 16,384-bubble local model, current build vs ab/lm_old (local_model.cpp before round 6's
# host changes), interleaved on the same box
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2 3; do for v in default lm_old; do
  if [ "$v" = default ]; then unset HDBMI_LIB; else export HDBMI_LIB=$PWD/ab/$v/libhdbmi.so; fi
  echo -n "$v "; timeout -k 10 300 python -u tools/lm_bench.py 16384 8 3 2>>"$OUT/stderr.log" | grep '"b"'
done; done > "$OUT/ab.log" 2>&1
cat "$OUT/ab.log"
