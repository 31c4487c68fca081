#!/bin/bash
# Profiles the C4 MFMA k-NN (tools/k1m_bench.py) on the GPU box: kernel stats at full size,
# SQ/GRBM PMC passes (MFMA busy cycles, wait/issue split, LDS) and FETCH/WRITE_SIZE at a
# reduced n, each pass a run of its own.
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
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d "$OUT/sq" -o k1m --output-format csv -- \
    python3 "$ROOT/tools/k1m_bench.py" "$NP" 128 > "$OUT/k1m_pmc.json.txt" 2> "$OUT/sq.err"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU -d "$OUT/lds" -o k1m --output-format csv -- \
    python3 "$ROOT/tools/k1m_bench.py" "$NP" 128 > /dev/null 2> "$OUT/lds.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o k1m --output-format csv -- \
    python3 "$ROOT/tools/k1m_bench.py" "$NP" 128 > /dev/null 2> "$OUT/fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o k1m --output-format csv -- \
    python3 "$ROOT/tools/k1m_bench.py" "$NP" 128 > /dev/null 2> "$OUT/write.err"
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/pmc_summary.json"
