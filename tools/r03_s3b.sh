# K1m screen cycle split (profiling build) + sharded-bubble driver tests and the C5 line
OUT=gpurun_out/s3b; mkdir -p $OUT; export TMPDIR=/tmp
HDBMI_LIB=$PWD/ab/k1_prof/libhdbmi.so K1M_QUICK=1 K1M_PROF=1 K1M_DIAG=1 timeout -k 10 200 python -u tools/k1m_bench.py 2000000 128 > $OUT/k1m_prof.json 2>&1 || { echo "k1m prof failed"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_driver.py tests/test_gpu_sharded.py tests/test_gpu_mr_scaled.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python -u bench.py --workload c5 --phases --no-cpu-baseline > $OUT/bench_c5.json.log 2>&1 || { echo "c5 failed"; exit 1; }
echo done
