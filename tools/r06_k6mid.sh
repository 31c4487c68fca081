#!/bin/bash
# K6 dc_mid (round 6): flat-label tests, then flat_mid_log A/B on the 1M C2 partition, then a
# one-partition rocprof of the default
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_ssort.py -x -q --timeout 300 --timeout-method thread -k "flat" > "$OUT/t_flat.log" 2>&1 || { echo "flat tests failed"; tail -40 "$OUT/t_flat.log"; exit 1; }
tail -2 "$OUT/t_flat.log"
for r in 1 2; do for v in 0 12 13 14 15; do echo -n "mid=$v "; HDB_FLAT_MID=$v timeout -k 10 200 python -u tools/c2_part.py 5 2>>"$OUT/stderr.log" | tail -1; done; done > "$OUT/ab.log" 2>&1
cat "$OUT/ab.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o part --output-format csv -- python3 tools/c2_part.py 5 > "$OUT/c2_prof.log" 2>&1 || { echo "prof failed"; tail -20 "$OUT/c2_prof.log"; exit 1; }
echo done
