#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# A/B of C2 builds (bench.py, default workload): each variant in its own process, interleaved.
# Usage: bash tools/ab_c2.sh <variant dir under ab/> ...
set -e
for r in $(seq 1 ${AB_REPS:-3}); do
for v in default "$@"; do
  if [ "$v" = default ]; then unset HDBMI_LIB; else export HDBMI_LIB=$PWD/ab/$v/libhdbmi.so; fi
  echo -n "$v "; timeout -k 10 200 python -u bench.py --no-cpu-baseline 2>>gpurun_out/tools_stderr.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['hbm_resident_ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_partition'].items()})"
done; done
