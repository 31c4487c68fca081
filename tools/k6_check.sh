mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# K6 check: flat-label GPU tests, the 1M timing, the C2 bench, and a kernel trace
mkdir -p gpurun_out/k6 && export TMPDIR=/tmp && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py -x -v --timeout 200 --timeout-method thread > gpurun_out/k6/test.log 2>&1 && \
for r in 1 2; do for lb in 9 10; do echo -n "lb=$lb "; HDB_FLAT_BLOCK_LOG=$lb timeout -k 10 120 python -u tools/flat_bench.py 1000000 20 2>>gpurun_out/tools_stderr.log | tail -1; done; done > gpurun_out/k6/bench.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/k6/c2.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/k6/trace -o ft --output-format csv -- python3 tools/flat_bench.py 1000000 3 > gpurun_out/k6/prof.log 2>&1; echo rc=$?
