#!/bin/bash
# C2 pipeline shapes (stage-1 MST workers x label workers), 40-step runs, two passes
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do for v in "5 2" "6 3" "5 3" "4 2" "6 2"; do set -- $v
  echo -n "mst=$1 label=$2 "; timeout -k 10 200 python -u bench.py --steps 40 --no-cpu-baseline --mst-workers $1 --label-workers $2 2>>"$OUT/stderr.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['hbm_resident_ms_per_step'],3), round(d['latency_ms_per_step'],3))"; done; done > "$OUT/shapes.log" 2>&1
cat "$OUT/shapes.log"
