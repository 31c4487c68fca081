#!/bin/bash
# round 6 closing profiles (call 1 of 2): C2 rocprof stats + PMC passes (tools/profile_bench.sh),
# C4 stats + PMC (tools/c4prof.sh), and a one-partition C2 kernel split (tools/c2_part.py).
# The PMC summaries are copied into profiles/r06/ before the closing lines (call 2) run, so each
# line's roofline.traffic reads the summary of the same build.
# Usage (repo root, on the box): bash tools/r06_final_prof.sh <outdir>
set -uo pipefail
mkdir -p "${1:?outdir}"; OUT=$(readlink -f "$1"); export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8  # as bench.py sets it (the profiler initialises HIP before bench.py runs)
timeout -k 10 700 bash tools/profile_bench.sh "$OUT/prof_c2" > "$OUT/prof_c2.log" 2>&1 || { echo "c2 profile failed"; tail "$OUT/prof_c2.log"; exit 1; }
timeout -k 10 600 bash tools/c4prof.sh "$OUT/c4_prof" > "$OUT/c4_prof.log" 2>&1 || { echo "c4 profile failed"; tail "$OUT/c4_prof.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/part" -o part --output-format csv -- python3 tools/c2_part.py 5 > "$OUT/part.log" 2>&1 || { echo "part profile failed"; exit 1; }
echo done
