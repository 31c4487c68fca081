#!/bin/bash
# round 4 check D: K2b row-batched leaf groups -- parity (tree, parity, C1), cycle split, C2 A/B
set -uo pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_c1.py tests/test_gpu_mr_scaled.py -x -q --timeout 300 --timeout-method thread -k "not full_size_partitioned" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
HDBMI_LIB=$PWD/ab/borprof/libhdbmi.so timeout -k 10 200 python -u tools/boruvka_stats.py > $OUT/borprof.log 2>&1 || { echo "borprof failed"; tail -20 $OUT/borprof.log; exit 1; }
AB_REPS=2 timeout -k 10 700 bash tools/ab_c2.sh rows0 rows8 rows64 > $OUT/ab_c2.log 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_c2.log; exit 1; }
echo done
