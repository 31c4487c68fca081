#!/bin/bash
# Round-end check on the GPU box: full GPU test suite, smoke(), default bench, C2 profile
# (kernel stats + PMC passes).  Usage (repo root, on the box): bash tools/round_check.sh <outdir>
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gputest.log" 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python bench.py > "$OUT/bench_c2.json.log" 2>&1 || { echo "bench failed"; exit 1; }
timeout -k 10 600 bash tools/profile_bench.sh "$OUT/prof_c2" > "$OUT/prof_c2.log" 2>&1 || { echo "profile failed"; exit 1; }
echo done
