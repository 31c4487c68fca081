#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# A/B of C4 builds (bench.py --workload c4): each variant in its own process, interleaved.
# Usage: bash tools/ab_c4.sh <variant dir under ab/> ...
set -e
for r in $(seq 1 ${AB_REPS:-2}); do
for v in default "$@"; do
  if [ "$v" = default ]; then unset HDBMI_LIB; else export HDBMI_LIB=$PWD/ab/$v/libhdbmi.so; fi
  echo -n "$v "; timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline 2>>gpurun_out/tools_stderr.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['ms_per_step'],2), 'hbm', round(d.get('hbm_resident_ms_per_step',0),2), 'screen', round(r['kernel_s_per_step']*1e3,2), 'order', round(r['order_s_per_step']*1e3,2), 'final', round(r['recheck_s_per_step']*1e3,2))"
done; done
