#!/bin/bash
# label-stage stream priority (HDB_BENCH_STAGE2_PRIO 0 / -1) on the final build, 20 steps, 5 runs
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2 3 4 5; do for p in 0 -1; do
  echo -n "prio=$p "; HDB_BENCH_STAGE2_PRIO=$p timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 2>>"$OUT/stderr.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3))"
done; done > "$OUT/ab.log" 2>&1
python3 - "$OUT/ab.log" <<'PY'
import sys, collections, statistics
v = collections.defaultdict(list)
for l in open(sys.argv[1]):
    p = l.split()
    if len(p) == 2: v[p[0]].append(float(p[1]))
for k, xs in v.items():
    print(k, "median %.3f ms/step" % statistics.median(xs), xs)
PY
