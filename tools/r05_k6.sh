#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# K6 check: flat-label tests + per-partition profile, flat_relabel A/B on the 1M merged list
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_c1.py -x -v --timeout 300 --timeout-method thread > "$OUT/t_flat.log" 2>&1 || { echo "flat tests failed"; tail -40 "$OUT/t_flat.log"; exit 1; }
for r in 1 2; do for v in 1 0; do echo -n "relabel=$v "; HDB_FLAT_RELABEL=$v timeout -k 10 200 python -u tools/c2_part.py 5 2>>gpurun_out/tools_stderr.log | tail -1; done; done > "$OUT/ab.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o part --output-format csv -- python3 tools/c2_part.py 4 > "$OUT/c2_prof.log" 2>&1 || { echo "prof failed"; tail -20 "$OUT/c2_prof.log"; exit 1; }
echo done
