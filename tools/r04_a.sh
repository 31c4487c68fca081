#!/bin/bash
# round 4 check A: K2b cycle split + cooperative Prim phases (profiling builds), the changed GPU
# tests (flat long chains, full-size C4, sharded world 3/4, merged-order leaf), then the C2 and
# C4 bench lines with the H2D-inclusive value
set -uo pipefail
OUT=gpurun_out/r04a; mkdir -p $OUT; export TMPDIR=/tmp
HDBMI_LIB=$PWD/ab/borprof/libhdbmi.so timeout -k 10 200 python -u tools/boruvka_stats.py > $OUT/borprof.log 2>&1 || { echo "borprof failed"; tail -20 $OUT/borprof.log; exit 1; }
HDBMI_LIB=$PWD/ab/coopprof/libhdbmi.so timeout -k 10 200 python -u tools/coop_prof.py 16384 8 > $OUT/coopprof.log 2>&1 || { echo "coopprof failed"; tail -20 $OUT/coopprof.log; exit 1; }
for bs in 1024 512 0; do HDB_PRIM_COOP_BS=$bs timeout -k 10 120 python -u tools/prim_xcd_bench.py 16384 8 > $OUT/prim_bs$bs.log 2>&1 || { echo "prim bs $bs failed"; tail -20 $OUT/prim_bs$bs.log; exit 1; }; done
for bs in 1024 0; do HDB_PRIM_COOP_BS=$bs timeout -k 10 120 python -u tools/prim_xcd_bench.py 4096 16 > $OUT/prim4k_bs$bs.log 2>&1 || { echo "prim4k bs $bs failed"; exit 1; }; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_flat.py tests/test_gpu_mfma.py tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
timeout -k 10 300 python -u bench.py > $OUT/bench_c2.json.log 2>&1 || { echo "bench c2 failed"; tail -20 $OUT/bench_c2.json.log; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4 > $OUT/bench_c4.json.log 2>&1 || { echo "bench c4 failed"; tail -20 $OUT/bench_c4.json.log; exit 1; }
echo done
