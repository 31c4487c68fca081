# round-3 batch: dc_root A/B (tests + timings), CreateLocalMST record tests, C5 with phases
# (per-task durations -> predicted scaling)
mkdir -p gpurun_out/k6ab gpurun_out/c5 && export TMPDIR=/tmp && \
timeout -k 10 300 python -u -m pytest tests/test_formats.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/k6ab/test_formats.log 2>&1 && \
for v in 3 4 5; do HDB_FLAT_ROOT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py -x -q --timeout 200 --timeout-method thread > gpurun_out/k6ab/test_v$v.log 2>&1 || exit 1; done && \
for r in 1 2; do for v in 0 1 3 4 5; do echo -n "root=$v "; HDB_FLAT_ROOT=$v timeout -k 10 120 python -u tools/flat_bench.py 1000000 20 2>/dev/null | tail -1; done; done > gpurun_out/k6ab/bench.log 2>&1 && \
timeout -k 10 400 python -u bench.py --workload c5 --phases --no-cpu-baseline > gpurun_out/c5/c5_phases.log 2>&1; echo rc=$?
