#!/bin/bash
# K2b knob re-sweep on the round-6 build (ab/ variants): one-partition scan time, 3 interleaved runs
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; shift; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2 3; do for v in default "$@"; do
  if [ "$v" = default ]; then unset HDBMI_LIB; else export HDBMI_LIB=$PWD/ab/$v/libhdbmi.so; fi
  echo -n "$v "; timeout -k 10 200 python -u tools/c2_part.py 5 2>>"$OUT/stderr.log" | tail -1
done; done > "$OUT/part.log" 2>&1
python3 - "$OUT/part.log" <<'PY'
import ast, collections, statistics, sys
v = collections.defaultdict(list)
for l in open(sys.argv[1]):
    k = l.split()[0]
    d = ast.literal_eval(l[l.index("{"):])
    v[k].append(d["boruvka_scan"])
for k, xs in v.items():
    print(k, "scan median %.3f ms (n=%d)" % (statistics.median(xs), len(xs)))
PY
