#!/bin/bash
# full GPU suite + smoke on the current build (one pytest process), then the closing profiles
# (tools/r06_final_prof.sh).  Usage: bash tools/r06_suite.sh <outdir>
mkdir -p gpurun_out
set -uo pipefail
mkdir -p "${1:?outdir}"; OUT=$(readlink -f "$1"); export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_full.log" 2>&1 || { echo "suite failed"; tail -30 "$OUT/pytest_full.log"; exit 1; }
tail -1 "$OUT/pytest_full.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
bash tools/r06_final_prof.sh "$OUT/final" || exit 1
