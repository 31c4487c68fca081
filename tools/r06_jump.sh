#!/bin/bash
# K6 pointer-jumping grid caps (ab/jump512, ab/jump256 vs default): flat tests on jump256,
# per-partition flat-labels time, jump kernel times from one trace each
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
HDBMI_LIB=$PWD/ab/jump256/libhdbmi.so timeout -k 10 600 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_ssort.py -x -q --timeout 300 --timeout-method thread -k "flat" > "$OUT/t_flat.log" 2>&1 || { echo "flat tests failed"; tail -40 "$OUT/t_flat.log"; exit 1; }
tail -1 "$OUT/t_flat.log"
for r in 1 2 3; do for v in default jump512 jump256; do
  if [ "$v" = default ]; then unset HDBMI_LIB; else export HDBMI_LIB=$PWD/ab/$v/libhdbmi.so; fi
  echo -n "$v "; timeout -k 10 200 python -u tools/c2_part.py 5 2>>"$OUT/stderr.log" | tail -1
done; done > "$OUT/part.log" 2>&1
unset HDBMI_LIB
cat "$OUT/part.log"
for v in default jump256; do
  if [ "$v" = default ]; then unset HDBMI_LIB; else export HDBMI_LIB=$PWD/ab/$v/libhdbmi.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/st_$v" -o p --output-format csv -- python3 tools/c2_part.py 5 > /dev/null 2>&1 || echo "prof failed"
  python3 - "$OUT/st_$v" $v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    tot = 0.0
    for r in csv.DictReader(open(f)):
        if any(k in r["Name"] for k in ("fl_jump(", "fo_jump_sum", "fo_sel_jump")):
            tot += float(r["TotalDurationNs"])
            print(sys.argv[2], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
    print(sys.argv[2], "jump kernels per partition us", round(tot / 6 / 1e3, 1))
PY
done
