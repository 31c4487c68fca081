#!/bin/bash
# K1t rows with lane shuffles instead of LDS (occupancy): builds under ab/ (HDBMI_LIB), tree tests on
# the 8-wave build, per-partition and pipelined A/B, kernel resources from one trace
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
HDBMI_LIB=$PWD/ab/k1t_shfl8/libhdbmi.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py -x -q --timeout 300 --timeout-method thread > "$OUT/t_tree.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/t_tree.log"; exit 1; }
tail -1 "$OUT/t_tree.log"
for r in 1 2 3; do for v in default k1t_shfl5 k1t_shfl6 k1t_shfl8; do
  if [ "$v" = default ]; then unset HDBMI_LIB; else export HDBMI_LIB=$PWD/ab/$v/libhdbmi.so; fi
  echo -n "$v "; timeout -k 10 200 python -u tools/c2_part.py 5 2>>"$OUT/stderr.log" | tail -1
done; done > "$OUT/part.log" 2>&1
unset HDBMI_LIB
cat "$OUT/part.log"
AB_REPS=3 bash tools/ab_c2.sh k1t_shfl6 k1t_shfl8 > "$OUT/bench.log" 2>&1; cat "$OUT/bench.log"
HDBMI_LIB=$PWD/ab/k1t_shfl8/libhdbmi.so timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/tr" -o p --output-format csv -- python3 tools/c2_part.py 1 > /dev/null 2>&1 || echo "trace failed"
python3 - "$OUT/tr" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "knn_tree_kernel" in r["Kernel_Name"]:
            print("knn_tree LDS", r["LDS_Block_Size"], "VGPR", r["VGPR_Count"], "scratch", r["Scratch_Size"]); break
PY
