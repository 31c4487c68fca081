#!/bin/bash
# pipelined C2 bench medians: default build vs ab/<variant> (5 interleaved runs each)
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; V=${2:?variant}; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2 3 4 5; do for v in default "$V"; do
  if [ "$v" = default ]; then unset HDBMI_LIB; else export HDBMI_LIB=$PWD/ab/$v/libhdbmi.so; fi
  echo -n "$v "; timeout -k 10 200 python -u bench.py --no-cpu-baseline 2>>"$OUT/stderr.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['hbm_resident_ms_per_step'],3), round(d['latency_ms_per_step'],3), round(d['kernels_ms_per_partition']['knn_tree'],3))"
done; done > "$OUT/ab.log" 2>&1
python3 - "$OUT/ab.log" <<'PY'
import sys, collections, statistics
v = collections.defaultdict(list)
for l in open(sys.argv[1]):
    p = l.split()
    if len(p) >= 5: v[p[0]].append([float(x) for x in p[1:5]])
for k, xs in v.items():
    print(k, "median ms/step %.3f hbm %.3f latency %.3f k1t %.3f (n=%d)" % tuple([statistics.median(x[i] for x in xs) for i in range(4)] + [len(xs)]))
PY
