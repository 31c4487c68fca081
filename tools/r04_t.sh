#!/bin/bash
# K2b/K1t rows-path thresholds (C2 A/B), then C5 model threads 6 / 8 / 4
set -o pipefail
mkdir -p gpurun_out/r04t
AB_REPS=3 bash tools/ab_c2.sh rm8 rm32 rm64 krm32 > gpurun_out/r04t/ab_c2.log 2>&1 || exit 1
for r in 1 2; do for t in 6 8 4; do
  echo -n "threads $t "; HDB_MODEL_THREADS=$t timeout -k 10 200 python -u bench.py --workload c5 --phases --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['predicted_scaling']['phases']['1']; print(round(d['ms_per_step']/1e3,3), 's', {k: round(v,3) for k,v in p.items()})"
done; done > gpurun_out/r04t/threads.log 2>&1
echo done
