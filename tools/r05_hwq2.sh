#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# finer C2 sweep over hardware queues x pipeline shape, then C5 at 4 vs 8 queues
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do for v in "8 5 2" "8 4 2" "8 5 3" "12 5 2" "12 6 2" "8 4 1"; do set -- $v
  echo -n "hwq=$1 mst=$2 label=$3 "; HDB_HW_QUEUES=$1 timeout -k 10 200 python -u bench.py --steps 40 --no-cpu-baseline --mst-workers $2 --label-workers $3 2>>gpurun_out/tools_stderr.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['hbm_resident_ms_per_step'],3), round(d['latency_ms_per_step'],3))"
done; done > "$OUT/hwq2.log" 2>&1
cat "$OUT/hwq2.log"
for q in 4 8; do echo -n "c5 hwq=$q "; HDB_HW_QUEUES=$q timeout -k 10 400 python -u bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline 2>>gpurun_out/tools_stderr.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],1), d.get('predicted_scaling',{}).get('speedup'))"; done > "$OUT/c5.log" 2>&1
cat "$OUT/c5.log"
