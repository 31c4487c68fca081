#!/bin/bash
# K2b scan rows with lane shuffles instead of LDS (occupancy): tree tests on the shuffle build,
# per-partition A/B, pipelined medians, kernel resources
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
HDBMI_LIB=$PWD/ab/bor_shfl4/libhdbmi.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py -x -q --timeout 300 --timeout-method thread > "$OUT/t_tree.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/t_tree.log"; exit 1; }
tail -1 "$OUT/t_tree.log"
for r in 1 2 3; do for v in default bor_shfl4 bor_shfl6; do
  if [ "$v" = default ]; then unset HDBMI_LIB; else export HDBMI_LIB=$PWD/ab/$v/libhdbmi.so; fi
  echo -n "$v "; timeout -k 10 200 python -u tools/c2_part.py 5 2>>"$OUT/stderr.log" | tail -1
done; done > "$OUT/part.log" 2>&1
unset HDBMI_LIB
cat "$OUT/part.log"
bash tools/r06_ab5.sh "$OUT/ab4" bor_shfl4 > /dev/null 2>&1; tail -2 "$OUT/ab4/ab.log" > /dev/null
python3 - "$OUT/ab4/ab.log" <<'PY'
import sys, collections, statistics
v = collections.defaultdict(list)
for l in open(sys.argv[1]):
    p = l.split()
    if len(p) >= 5: v[p[0]].append([float(x) for x in p[1:5]])
for k, xs in v.items():
    print(k, "median ms/step %.3f hbm %.3f latency %.3f k1t %.3f (n=%d)" % tuple([statistics.median(x[i] for x in xs) for i in range(4)] + [len(xs)]))
PY
for v in bor_shfl4 bor_shfl6; do
HDBMI_LIB=$PWD/ab/$v/libhdbmi.so timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/tr_$v" -o p --output-format csv -- python3 tools/c2_part.py 1 > /dev/null 2>&1 || echo "trace failed"
python3 - "$OUT/tr_$v" $v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "boruvka_bvh_kernel" in r["Kernel_Name"]:
            print(sys.argv[2], "boruvka_bvh LDS", r["LDS_Block_Size"], "VGPR", r["VGPR_Count"], "scratch", r["Scratch_Size"]); break
PY
done
