#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# K1m screen cycle split (HDB_K1S_PROF build) at C4
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/k1m_bench.py > "$OUT/default.json" 2>>gpurun_out/tools_stderr.log || exit 1
K1M_QUICK=1 K1M_PROF=1 K1M_DIAG=1 HDBMI_LIB=$PWD/ab/k1prof/libhdbmi.so timeout -k 10 300 python -u tools/k1m_bench.py > "$OUT/prof.json" 2>>gpurun_out/tools_stderr.log || exit 1
cat "$OUT"/*.json
