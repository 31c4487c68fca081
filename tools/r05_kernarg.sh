#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# C2 line (and its unpipelined latency) with and without HIP_FORCE_DEV_KERNARG=1
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do for v in 0 1; do
  echo -n "dev_kernarg=$v "; HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python -u bench.py --steps 40 --no-cpu-baseline 2>>gpurun_out/tools_stderr.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['hbm_resident_ms_per_step'],3), round(d['latency_ms_per_step'],3), d['kernels_ms_per_partition'])"
done; done > "$OUT/kernarg.log" 2>&1
cat "$OUT/kernarg.log"
