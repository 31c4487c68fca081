#!/bin/bash
# K2b scan XCD-interleaved chunks (HDB_BOR_XCD chunks per XCD): tree tests, per-partition A/B,
# pipelined bench A/B, FETCH_SIZE per variant
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py -x -q --timeout 300 --timeout-method thread > "$OUT/t_tree.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/t_tree.log"; exit 1; }
tail -1 "$OUT/t_tree.log"
for r in 1 2 3; do for x in 0 4 8 16; do
  echo -n "m=$x "; HDB_BOR_XCD=$x timeout -k 10 200 python -u tools/c2_part.py 5 2>>"$OUT/stderr.log" | tail -1
done; done > "$OUT/part.log" 2>&1
cat "$OUT/part.log"
for r in 1 2 3; do for x in 0 8; do
  echo -n "m=$x "; HDB_BOR_XCD=$x timeout -k 10 200 python -u bench.py --no-cpu-baseline 2>>"$OUT/stderr.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['hbm_resident_ms_per_step'],3), round(d['latency_ms_per_step'],3), d['kernels_ms_per_partition'])"
done; done > "$OUT/bench.log" 2>&1
cat "$OUT/bench.log"
for x in 0 8; do
  HDB_BOR_XCD=$x timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch$x" -o p --output-format csv -- python3 tools/c2_part.py 2 > /dev/null 2>> "$OUT/stderr.log" || { echo "pmc $x failed"; exit 1; }
  python3 - "$OUT/fetch$x" "$x" <<'PY'
import csv, glob, sys
v = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(f)) if "boruvka_bvh_kernel" in r["Kernel_Name"]]
print("m=%s boruvka_bvh FETCH_SIZE x2 per launch: %.1f MB over %d launches" % (sys.argv[2], 2 * 1024 * sum(v) / max(len(v), 1) / 1e6, len(v)))
PY
done
