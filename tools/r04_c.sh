#!/bin/bash
# round 4 check C: cooperative Prim phases / caching / slots A/B, C4 re-check A/B, C2 + C4 bench lines
set -uo pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT; export TMPDIR=/tmp
HDBMI_LIB=$PWD/ab/coopprof/libhdbmi.so timeout -k 10 120 python -u tools/coop_prof.py 16384 8 > $OUT/coopprof.log 2>&1 || { echo "coopprof failed"; exit 1; }
BUBBLES=1 HDBMI_LIB=$PWD/ab/coopprof/libhdbmi.so timeout -k 10 120 python -u tools/coop_prof.py 16384 8 > $OUT/coopprof_bubbles.log 2>&1 || { echo "coopprof b failed"; exit 1; }
timeout -k 10 120 python -u tools/prim_xcd_bench.py 16384 8 > $OUT/prim16k.log 2>&1 || { echo "prim bench failed"; exit 1; }
HDBMI_LIB=$PWD/ab/nocache/libhdbmi.so timeout -k 10 120 python -u tools/prim_xcd_bench.py 16384 8 > $OUT/prim16k_nocache.log 2>&1 || { echo "prim bench nocache failed"; exit 1; }
HDB_PRIM_COOP_SLOTS=5 timeout -k 10 120 python -u tools/prim_xcd_bench.py 16384 8 > $OUT/prim16k_slots5.log 2>&1 || { echo "prim bench slots5 failed"; exit 1; }
timeout -k 10 200 python -u tools/bubble_stats_bench.py > $OUT/bubble_stats.log 2>&1 || { echo "bubble bench failed"; tail -20 $OUT/bubble_stats.log; exit 1; }
AB_REPS=2 timeout -k 10 600 bash tools/ab_c4.sh k1f16 k1fpf2 > $OUT/ab_c4.log 2>&1 || { echo "ab c4 failed"; tail -20 $OUT/ab_c4.log; exit 1; }
echo done
