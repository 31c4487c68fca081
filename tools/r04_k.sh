#!/bin/bash
# round 4 check K: wider C2 pipeline shapes (40 timed steps); K1m re-check prefetch width A/B
set -uo pipefail
OUT=gpurun_out/r04k; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
for cfg in "5 3" "6 3" "6 4" "7 3" "8 4" "5 2"; do
  set -- $cfg
  echo -n "mst $1 label $2: " >> $OUT/workers.log
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 --warmup 5 --mst-workers $1 --label-workers $2 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['hbm_resident_ms_per_step'],3))" >> $OUT/workers.log || { echo "bench failed"; exit 1; }
done; done
AB_REPS=2 timeout -k 10 500 bash tools/ab_c4.sh k1fu32 k1fu8 > $OUT/ab_c4.log 2>&1 || { echo "ab c4 failed"; exit 1; }
echo done
