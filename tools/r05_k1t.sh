#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# K1t XCD-local dynamic tile order: tree/knn tests, then one-partition A/B (ab/k1tstat = static order)
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_c1.py -x -q --timeout 300 --timeout-method thread > "$OUT/t.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/t.log"; exit 1; }
tail -1 "$OUT/t.log"
for r in 1 2 3; do for v in default k1tstat; do
  if [ "$v" = default ]; then unset HDBMI_LIB; else export HDBMI_LIB=$PWD/ab/$v/libhdbmi.so; fi
  echo -n "$v "; timeout -k 10 200 python -u tools/c2_part.py 5 2>>gpurun_out/tools_stderr.log | tail -1
done; done > "$OUT/ab.log" 2>&1
cat "$OUT/ab.log"
