#!/bin/bash
# Profiles bench.py on the GPU box: kernel-trace stats pass, then one PMC pass per TCC
# counter (FETCH_SIZE and WRITE_SIZE do not fit one pass), then a per-kernel byte summary.
# Usage (from the repo root, on the box): bash tools/profile_bench.sh <outdir> [bench args]
set -euo pipefail
OUT=$(readlink -f "${1:?outdir}")
shift
ARGS=("$@")
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o bench --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline "${ARGS[@]}" > "$OUT/bench.json.log" 2> "$OUT/stats.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o bench --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "${ARGS[@]}" > /dev/null 2> "$OUT/fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o bench --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "${ARGS[@]}" > /dev/null 2> "$OUT/write.err"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -d "$OUT/sq" -o bench --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "${ARGS[@]}" > /dev/null 2> "$OUT/sq.err"
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/pmc_summary.json"
