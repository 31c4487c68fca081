# K2b scan diagnostics: per-round stats (visits, waves, wave-cycle tail) and one SQ PMC pass
mkdir -p gpurun_out/k2b && export TMPDIR=/tmp && \
timeout -k 10 200 python -u tools/boruvka_stats.py > gpurun_out/k2b/stats.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_WAIT_ANY -d gpurun_out/k2b/sq -o k2b --output-format csv -- python3 tools/boruvka_stats.py > gpurun_out/k2b/sq.log 2>&1; echo rc=$?
