#!/bin/bash
# ssort micro-benchmark: wall, kernel stats, SQ counters of the sample-sort kernels
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/ssort_bench.py 20 > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o ss --output-format csv -- python3 tools/ssort_bench.py 10 > "$OUT/prof.log" 2>&1 || { echo "prof failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$OUT/pmc" -o ss --output-format csv -- python3 tools/ssort_bench.py 2 > "$OUT/pmc.log" 2>&1 || { echo "pmc failed"; exit 1; }
echo done
