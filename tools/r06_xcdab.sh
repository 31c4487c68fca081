#!/bin/bash
# pipelined C2 bench: K1t / K2b-scan XCD chunks on and off (HDB_K1T_XCD / HDB_BOR_XCD), interleaved
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2 3 4 5; do for cfg in "0 0" "8 8" "8 0" "0 8"; do set -- $cfg
  echo -n "k1t=$1 bor=$2 "; HDB_K1T_XCD=$1 HDB_BOR_XCD=$2 timeout -k 10 200 python -u bench.py --no-cpu-baseline 2>>"$OUT/stderr.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['hbm_resident_ms_per_step'],3), round(d['latency_ms_per_step'],3))"
done; done > "$OUT/ab.log" 2>&1
python3 - "$OUT/ab.log" <<'PY'
import sys, collections, statistics
v = collections.defaultdict(list)
for l in open(sys.argv[1]):
    p = l.split()
    if len(p) >= 5: v[(p[0], p[1])].append((float(p[2]), float(p[3]), float(p[4])))
for k, xs in v.items():
    print(k, "ms/step median %.3f  hbm %.3f  latency %.3f  (n=%d)" % tuple([statistics.median(x[i] for x in xs) for i in range(3)] + [len(xs)]))
PY
