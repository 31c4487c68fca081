#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# A/B of C5 builds (bench.py --workload c5 --phases): whole-job seconds and the nearest-sample phase.
# Usage: bash tools/ab_c5.sh <variant dir under ab/> ...
set -e
for r in $(seq 1 ${AB_REPS:-1}); do
for v in default "$@"; do
  if [ "$v" = default ]; then unset HDBMI_LIB; else export HDBMI_LIB=$PWD/ab/$v/libhdbmi.so; fi
  echo -n "$v "; timeout -k 10 200 python -u bench.py --workload c5 --phases --no-cpu-baseline 2>>gpurun_out/tools_stderr.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['predicted_scaling']['phases']['1']; print(round(d['ms_per_step']/1e3,3), 's', {k: round(v,3) for k,v in p.items()})"
done; done
