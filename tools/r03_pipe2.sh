# C2 pipeline with H2D prefetch: stage-2 stream priority A/B (0 = normal, -1 = high), alternated
mkdir -p gpurun_out/pipe2 && export TMPDIR=/tmp && \
timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/pipe2/p0a.json.log 2>&1 && \
HDB_BENCH_STAGE2_PRIO=-1 timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/pipe2/p1a.json.log 2>&1 && \
timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/pipe2/p0b.json.log 2>&1 && \
HDB_BENCH_STAGE2_PRIO=-1 timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/pipe2/p1b.json.log 2>&1; echo rc=$?
