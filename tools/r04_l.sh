#!/bin/bash
# K2b leaf-batched rows: parity (tree tests), per-round times, C2 A/B vs the per-group rows
set -o pipefail
mkdir -p gpurun_out/r04l
timeout -k 10 400 python -u -m pytest tests/test_gpu_tree.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04l/tests.log 2>&1 || { echo tests failed; exit 1; }
for v in default lp0; do
  if [ "$v" = default ]; then unset HDBMI_LIB; else export HDBMI_LIB=$PWD/ab/$v/libhdbmi.so; fi
  timeout -k 10 200 python -u tools/boruvka_stats.py > gpurun_out/r04l/stats_$v.log 2>&1 || exit 1
done
unset HDBMI_LIB
AB_REPS=3 bash tools/ab_c2.sh lp0 pair0 lp2 > gpurun_out/r04l/ab_c2.log 2>&1
echo done
