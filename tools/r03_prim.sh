# cooperative Prim same-XCD exchange: step cost A/B + identical edges, Prim parity tests, C5 with it
mkdir -p gpurun_out/prim && export TMPDIR=/tmp && \
timeout -k 10 200 python -u tools/prim_xcd_bench.py 16384 8 > gpurun_out/prim/xcd_16k.log 2>&1 && \
timeout -k 10 200 python -u tools/prim_xcd_bench.py 4096 16 > gpurun_out/prim/xcd_4k.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_driver.py -x -q --timeout 300 --timeout-method thread > gpurun_out/prim/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c5 --phases --no-cpu-baseline > gpurun_out/prim/c5.log 2>&1 && \
HDB_PRIM_XCD=0 timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > gpurun_out/prim/c5_noxcd.log 2>&1; echo rc=$?
