#!/bin/bash
# round 4 check I: K1t XCD-contiguous tiles A/B; cooperative Prim workgroup size with caching
set -uo pipefail
OUT=gpurun_out/r04i; mkdir -p $OUT; export TMPDIR=/tmp
for bs in 1024 512 0; do HDB_PRIM_COOP_BS=$bs timeout -k 10 120 python -u tools/prim_xcd_bench.py 16384 8 > $OUT/prim_bs$bs.log 2>&1 || { echo "prim bs $bs failed"; exit 1; }; done
for bs in 1024 0; do HDB_PRIM_COOP_BS=$bs timeout -k 10 120 python -u tools/prim_xcd_bench.py 65536 8 > $OUT/prim64k_bs$bs.log 2>&1 || { echo "prim64k bs $bs failed"; exit 1; }; done
AB_REPS=2 timeout -k 10 500 bash tools/ab_c2.sh k1txcd > $OUT/ab_c2.log 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_c2.log; exit 1; }
echo done
