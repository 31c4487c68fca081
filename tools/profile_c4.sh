#!/bin/bash
# HBM traffic of the C4 line's kernels at full size: FETCH_SIZE and WRITE_SIZE passes (one
# run each) over bench.py --workload c4, then the per-kernel byte summary that bench.py's C4
# roofline reads as `traffic`.  Usage (repo root, on the box): bash tools/profile_c4.sh <outdir>
set -euo pipefail
OUT=$(readlink -f "${1:?outdir}")
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o c4 --output-format csv -- \
    python3 "$ROOT/bench.py" --workload c4 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> "$OUT/fetch.err"
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o c4 --output-format csv -- \
    python3 "$ROOT/bench.py" --workload c4 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> "$OUT/write.err"
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/pmc_summary.json"
