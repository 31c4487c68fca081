#!/bin/bash
# round 4 check B: two-pass leaf groups in K2b/K1t -- parity tests, K2b cycle split, C2 A/B vs the one-pass build
set -uo pipefail
OUT=gpurun_out/r04b; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
HDBMI_LIB=$PWD/ab/borprof/libhdbmi.so timeout -k 10 200 python -u tools/boruvka_stats.py > $OUT/borprof.log 2>&1 || { echo "borprof failed"; tail -20 $OUT/borprof.log; exit 1; }
timeout -k 10 900 bash tools/ab_c2.sh onepass > $OUT/ab_c2.log 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_c2.log; exit 1; }
timeout -k 10 300 python -u bench.py > $OUT/bench_c2.json.log 2>&1 || { echo "bench c2 failed"; tail -20 $OUT/bench_c2.json.log; exit 1; }
HDBMI_LIB=$PWD/ab/coopprof/libhdbmi.so timeout -k 10 120 python -u tools/coop_prof.py 16384 8 > $OUT/coopprof.log 2>&1 || { echo "coopprof failed"; exit 1; }
BUBBLES=1 HDBMI_LIB=$PWD/ab/coopprof/libhdbmi.so timeout -k 10 120 python -u tools/coop_prof.py 16384 8 > $OUT/coopprof_bubbles.log 2>&1 || { echo "coopprof b failed"; exit 1; }
timeout -k 10 120 python -u tools/prim_xcd_bench.py 16384 8 > $OUT/prim16k.log 2>&1 || { echo "prim bench failed"; exit 1; }
HDBMI_LIB=$PWD/ab/nocache/libhdbmi.so timeout -k 10 120 python -u tools/prim_xcd_bench.py 16384 8 > $OUT/prim16k_nocache.log 2>&1 || { echo "prim bench nocache failed"; exit 1; }
HDB_PRIM_COOP_SLOTS=5 timeout -k 10 120 python -u tools/prim_xcd_bench.py 16384 8 > $OUT/prim16k_slots5.log 2>&1 || { echo "prim bench slots5 failed"; exit 1; }
timeout -k 10 900 bash tools/ab_c4.sh k1f16 k1fpf2 k1fpf6 > $OUT/ab_c4.log 2>&1 || { echo "ab c4 failed"; tail -20 $OUT/ab_c4.log; exit 1; }
echo done
