mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# K6 A/B: dc_root variants (HDB_FLAT_ROOT 0/1/2): GPU tests per variant, then interleaved 1M timings
mkdir -p gpurun_out/k6ab && export TMPDIR=/tmp && \
for v in 3 4 5; do HDB_FLAT_ROOT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py -x -q --timeout 200 --timeout-method thread > gpurun_out/k6ab/test_v$v.log 2>&1 || exit 1; done && \
for r in 1 2; do for v in 0 1 3 4 5; do echo -n "root=$v "; HDB_FLAT_ROOT=$v timeout -k 10 120 python -u tools/flat_bench.py 1000000 20 2>>gpurun_out/tools_stderr.log | tail -1; done; done > gpurun_out/k6ab/bench.log 2>&1; echo rc=$?
