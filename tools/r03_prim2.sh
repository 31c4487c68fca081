# same-XCD Prim: rotation + 64-workgroup spread A/B; flat tests (selection flag change); C5 per setting
mkdir -p gpurun_out/prim2 && export TMPDIR=/tmp && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_parity.py -x -q -k "flat or device or prim or coop" --timeout 200 --timeout-method thread > gpurun_out/prim2/tests.log 2>&1 && \
timeout -k 10 200 python -u tools/prim_xcd_bench.py 16384 8 > gpurun_out/prim2/xcd_16k.log 2>&1 && \
HDB_PRIM_XCD_MAX_WG=64 timeout -k 10 300 python -u tools/prim_xcd_bench.py 65536 4 > gpurun_out/prim2/xcd_64k.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > gpurun_out/prim2/c5_max32.log 2>&1 && \
HDB_PRIM_XCD_MAX_WG=64 timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > gpurun_out/prim2/c5_max64.log 2>&1; echo rc=$?
