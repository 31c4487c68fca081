#!/bin/bash
# round 4 check D: K2b defaults (one pass, no leaf publish) -- cycle split with atomic-free stats, C2 A/B
set -uo pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT; export TMPDIR=/tmp
HDBMI_LIB=$PWD/ab/borprof/libhdbmi.so timeout -k 10 200 python -u tools/boruvka_stats.py > $OUT/borprof.log 2>&1 || { echo "borprof failed"; tail -20 $OUT/borprof.log; exit 1; }
AB_REPS=2 timeout -k 10 900 bash tools/ab_c2.sh r3pub refr5 refr10 twopass > $OUT/ab_c2.log 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_c2.log; exit 1; }
echo done
