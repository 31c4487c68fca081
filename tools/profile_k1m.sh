#!/bin/bash
# Profiles the C4 MFMA k-NN (tools/k1m_bench.py) on the GPU box: kernel stats at full size,
# one SQ/GRBM PMC pass (MFMA busy cycles) and FETCH_SIZE at a reduced n.
# Usage (repo root, on the box): bash tools/profile_k1m.sh <outdir> [n_full] [n_pmc]
set -euo pipefail
OUT=$(readlink -f "${1:?outdir}")
NF=${2:-2000000}
NP=${3:-400000}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o k1m --output-format csv -- \
    python3 "$ROOT/tools/k1m_bench.py" "$NF" 128 > "$OUT/k1m_full.json.txt" 2> "$OUT/stats.err"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE -d "$OUT/sq" -o k1m --output-format csv -- \
    python3 "$ROOT/tools/k1m_bench.py" "$NP" 128 > "$OUT/k1m_pmc.json.txt" 2> "$OUT/sq.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o k1m --output-format csv -- \
    python3 "$ROOT/tools/k1m_bench.py" "$NP" 128 > /dev/null 2> "$OUT/fetch.err"
