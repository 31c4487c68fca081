#!/bin/bash
# round 4 check J: C2 pipeline shape (stage-1 workers x label stages), 40 timed steps each
set -uo pipefail
OUT=gpurun_out/r04j2; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
for cfg in "3 2" "4 2" "2 2" "5 3" "3 3" "4 4"; do
  set -- $cfg
  echo -n "mst $1 label $2: " >> $OUT/workers.log
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 --warmup 5 --mst-workers $1 --label-workers $2 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['hbm_resident_ms_per_step'],3))" >> $OUT/workers.log || { echo "bench failed"; exit 1; }
done; done
echo done
