#!/bin/bash
# pipeline shapes on the final build at the driver's 20 steps: stage-1 partitions in flight x
# label stages, interleaved, 3 runs each (medians)
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2 3; do for sh in "5 2" "4 2" "6 2" "5 3" "6 3" "4 1"; do set -- $sh
  echo -n "mst=$1 label=$2 "; timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --mst-workers $1 --label-workers $2 2>>"$OUT/stderr.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3))"
done; done > "$OUT/ab.log" 2>&1
python3 - "$OUT/ab.log" <<'PY'
import sys, collections, statistics
v = collections.defaultdict(list)
for l in open(sys.argv[1]):
    p = l.split()
    if len(p) == 3: v[(p[0], p[1])].append(float(p[2]))
for k, xs in sorted(v.items(), key=lambda kv: statistics.median(kv[1])):
    print(k, "median %.3f ms/step" % statistics.median(xs), xs)
PY
