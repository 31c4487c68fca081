#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# C2 line vs hardware queues per process (GPU_MAX_HW_QUEUES; the box exports 4) and pipeline shape
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}" > "$OUT/hwq.log"
for r in 1 2; do for v in "4 5 2" "8 5 2" "8 6 2" "8 7 3" "16 7 3"; do set -- $v
  echo -n "hwq=$1 mst=$2 label=$3 "; HDB_HW_QUEUES=$1 timeout -k 10 200 python -u bench.py --steps 40 --no-cpu-baseline --mst-workers $2 --label-workers $3 2>>gpurun_out/tools_stderr.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['hbm_resident_ms_per_step'],3), round(d['latency_ms_per_step'],3))"
done; done >> "$OUT/hwq.log" 2>&1
cat "$OUT/hwq.log"
