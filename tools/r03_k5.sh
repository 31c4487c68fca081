# K5 chunked bubble kNN: parity tests, timing A/B, C5 with it
mkdir -p gpurun_out/k5 && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "bubble or local_model or prim" --timeout 300 --timeout-method thread > gpurun_out/k5/tests.log 2>&1 && \
timeout -k 10 200 python -u tools/bubble_knn_bench.py 16384 8 > gpurun_out/k5/bench16k.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_mr_scaled.py tests/test_gpu_c1.py -x -q --timeout 300 --timeout-method thread > gpurun_out/k5/tests_mr.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > gpurun_out/k5/c5.log 2>&1; echo rc=$?
