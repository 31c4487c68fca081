#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# C2 pipeline shapes (stage-1 workers x label stages), 40 steps each, two passes
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do for s in "5 2" "6 2" "5 3" "4 2" "7 3"; do set -- $s
  echo -n "mst=$1 label=$2 "; timeout -k 10 200 python -u bench.py --steps 40 --no-cpu-baseline --mst-workers $1 --label-workers $2 2>>gpurun_out/tools_stderr.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['hbm_resident_ms_per_step'],3), round(d['latency_ms_per_step'],3))"
done; done > "$OUT/shapes.log" 2>&1
echo done
