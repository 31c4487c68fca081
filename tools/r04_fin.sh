#!/bin/bash
# round 4 closing check: full GPU suite, smoke(), the C2 / C4 / C5 bench lines.  Usage: bash tools/r04_fin.sh <outdir>
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gputest.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$OUT/gputest.log"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python -u bench.py > "$OUT/bench_c2.json.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench_c2.json.log"; exit 1; }
timeout -k 10 200 python -u bench.py --workload c4 > "$OUT/bench_c4.json.log" 2>&1 || { echo "bench c4 failed"; exit 1; }
timeout -k 10 200 python -u bench.py --workload c5 --phases > "$OUT/bench_c5.json.log" 2>&1 || { echo "bench c5 failed"; exit 1; }
echo done
