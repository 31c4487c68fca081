#!/bin/bash
# C2 pipelined bench at 8 / 12 / 16 / 24 hardware queues (interleaved), plus the stream -> queue
# map of one 16-queue run (rocprofv3 kernel trace)
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2 3; do for q in 8 12 16 24; do
  echo -n "q=$q "; HDB_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --no-cpu-baseline 2>>"$OUT/stderr.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['hbm_resident_ms_per_step'],3), round(d['latency_ms_per_step'],3), d['config']['hw_queues'])"
done; done > "$OUT/ab.log" 2>&1
cat "$OUT/ab.log"
HDB_HW_QUEUES=16 timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/tr16" -o b --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > "$OUT/tr16.log" 2>&1 || echo "trace failed"
