#!/bin/bash
# round 4 check H: tree/parity/sharded tests with the wave-aggregated publish default, K2b cycle
# split, then the bench lines + C2 profile (tools/r04_bench.sh)
set -uo pipefail
OUT=gpurun_out/r04h; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_mr_scaled.py -x -q --timeout 300 --timeout-method thread -k "not full_size_partitioned" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
HDBMI_LIB=$PWD/ab/borprof/libhdbmi.so timeout -k 10 200 python -u tools/boruvka_stats.py > $OUT/borprof.log 2>&1 || { echo "borprof failed"; tail -20 $OUT/borprof.log; exit 1; }
bash tools/r04_bench.sh $OUT || exit 1
echo done
