mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# K6 A/B: dc_link variants (HDB_FLAT_LINK 0/1): tests, interleaved 1M timings, trace of the default
mkdir -p gpurun_out/k6ab2 && export TMPDIR=/tmp && \
HDB_FLAT_LINK=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py -x -q --timeout 200 --timeout-method thread > gpurun_out/k6ab2/test_l1.log 2>&1 && \
for r in 1 2 3; do for v in 0 1; do echo -n "link=$v "; HDB_FLAT_LINK=$v timeout -k 10 120 python -u tools/flat_bench.py 1000000 20 2>>gpurun_out/tools_stderr.log | tail -1; done; done > gpurun_out/k6ab2/bench.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/k6ab2/trace -o ft --output-format csv -- python3 tools/flat_bench.py 1000000 3 > gpurun_out/k6ab2/prof.log 2>&1; echo rc=$?
