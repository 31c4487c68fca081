#!/bin/bash
# C2 line with the runtime's copy engines vs blit kernels for the pinned H2D / D2H copies
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do for v in default 1 0; do
  echo -n "sdma=$v "
  if [ "$v" = default ]; then timeout -k 10 200 python -u bench.py --steps 40 --no-cpu-baseline 2>>"$OUT/stderr.log"; else HSA_ENABLE_SDMA=$v timeout -k 10 200 python -u bench.py --steps 40 --no-cpu-baseline 2>>"$OUT/stderr.log"; fi | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['hbm_resident_ms_per_step'],3), round(d['latency_ms_per_step'],3))"; done; done > "$OUT/sdma.log" 2>&1
cat "$OUT/sdma.log"
HSA_ENABLE_SDMA=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats1" -o b --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || echo "prof failed"
grep -i copy "$OUT"/stats1/*kernel_stats.csv | cut -c1-120
