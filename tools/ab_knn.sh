#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# A/B of K1 builds in one box session: each variant in its own process, interleaved twice.
set -e
for r in 1 2; do
for v in default abbuild/us4 abbuild/q4u8; do
  if [ "$v" = default ]; then unset HDBMI_LIB; else export HDBMI_LIB=$PWD/$v/libhdbmi.so; fi
  echo -n "$v "; timeout -k 10 120 python -u tools/knn_bench.py 1000000 2>>gpurun_out/tools_stderr.log | tail -1
done; done
