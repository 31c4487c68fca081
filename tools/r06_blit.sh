#!/bin/bash
# which runtime path carries the C2 line's large pinned copies: blit kernels (copyBuffer on 256
# workgroups) or the copy engines; GPU_FORCE_BLIT_COPY_SIZE / GPU_BLIT_ENGINE_TYPE A/B
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in "GPU_FORCE_BLIT_COPY_SIZE=0" "GPU_BLIT_ENGINE_TYPE=1" "GPU_BLIT_ENGINE_TYPE=2" "ROC_P2P_SDMA_SIZE=0"; do
  echo "== $v"
  env $v timeout -k 10 120 python -u bench.py --steps 40 --no-cpu-baseline 2>>"$OUT/stderr.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['hbm_resident_ms_per_step'],3), round(d['latency_ms_per_step'],3))"
done > "$OUT/blit.log" 2>&1
cat "$OUT/blit.log"
GPU_FORCE_BLIT_COPY_SIZE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats0" -o b --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || echo "prof failed"
grep -i copy "$OUT"/stats0/*kernel_stats.csv | cut -c1-120
