#!/bin/bash
# C5 model-thread count A/B (HDB_MODEL_THREADS), two runs each
set -o pipefail
mkdir -p gpurun_out/r04s
for r in 1 2; do for t in 4 6 3; do
  echo -n "threads $t "; HDB_MODEL_THREADS=$t timeout -k 10 200 python -u bench.py --workload c5 --phases --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['predicted_scaling']['phases']['1']; print(round(d['ms_per_step']/1e3,3), 's', {k: round(v,3) for k,v in p.items()})"
done; done > gpurun_out/r04s/threads.log 2>&1
echo done
