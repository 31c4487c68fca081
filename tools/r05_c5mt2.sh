#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# C5: local-model threads x hardware queues, two passes
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do for v in "4 8" "8 12" "8 8"; do set -- $v
  HDB_MODEL_THREADS=$1 HDB_HW_QUEUES=$2 timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > "$OUT/c5_t$1_q$2_r$r.json.log" 2>>gpurun_out/tools_stderr.log || { echo c5 failed; exit 1; }
  tail -1 "$OUT/c5_t$1_q$2_r$r.json.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('threads $1 q$2', round(d['ms_per_step'],1))"; done; done
