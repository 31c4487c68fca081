#!/bin/bash
# ssort check: its tests + the sort/merge/tree/flat suites, then the per-partition profile
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ssort.py -x -v --timeout 300 --timeout-method thread > "$OUT/t_ssort.log" 2>&1 || { echo "ssort tests failed"; tail -40 "$OUT/t_ssort.log"; exit 1; }
timeout -k 10 200 python -u tools/c2_part.py 5 > "$OUT/c2_part.log" 2>&1 || { echo "c2_part failed"; tail -20 "$OUT/c2_part.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o part --output-format csv -- python3 tools/c2_part.py 4 > "$OUT/c2_prof.log" 2>&1 || { echo "prof failed"; tail -20 "$OUT/c2_prof.log"; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py tests/test_gpu_flat.py tests/test_gpu_c1.py -x -q --timeout 300 --timeout-method thread > "$OUT/t_rest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/t_rest.log"; exit 1; }
echo done
