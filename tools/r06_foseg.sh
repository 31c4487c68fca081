#!/bin/bash
# K6 FOSC segment walker (HDB_FLAT_FOSEG=1) vs fo_walk (0): flat tests both ways, per-partition
# A/B, per-launch walker times
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for x in 1 0; do
HDB_FLAT_FOSEG=$x timeout -k 10 600 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_ssort.py tests/test_gpu_c1.py -x -q --timeout 300 --timeout-method thread -k "flat or c1" > "$OUT/t_flat$x.log" 2>&1 || { echo "flat tests failed ($x)"; tail -40 "$OUT/t_flat$x.log"; exit 1; }
tail -1 "$OUT/t_flat$x.log"
done
for r in 1 2 3; do for x in 0 1; do
  echo -n "foseg=$x "; HDB_FLAT_FOSEG=$x timeout -k 10 200 python -u tools/c2_part.py 5 2>>"$OUT/stderr.log" | tail -1
done; done > "$OUT/part.log" 2>&1
cat "$OUT/part.log"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/tr" -o p --output-format csv -- python3 tools/c2_part.py 2 > /dev/null 2>&1 || echo "trace failed"
python3 - "$OUT/tr" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    ks = [r for r in csv.DictReader(open(f)) if "fo_walk" in r["Kernel_Name"]]
    print("fo_walk_seg launches (last partition, us):", [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1) for r in ks[-20:]])
PY
