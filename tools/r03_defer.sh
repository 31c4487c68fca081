# deferred leaves: driver / sharded / scaled-C5 GPU tests, then the C5 line with phases
OUT=gpurun_out/defer; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_driver.py tests/test_gpu_sharded.py tests/test_gpu_mr_scaled.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python -u bench.py --workload c5 --phases --no-cpu-baseline > $OUT/bench_c5.json.log 2>&1 || { echo "c5 failed"; exit 1; }
echo done
