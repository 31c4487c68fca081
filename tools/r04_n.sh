#!/bin/bash
# K1m re-check counters: SQ cycle split, L1/L2 request counts, HBM fetch (C4 bench, one step)
set -o pipefail
OUT=gpurun_out/r04n; mkdir -p $OUT; export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $OUT/sq -o c4 --output-format csv -- \
  python3 bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/sq.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d $OUT/mem -o c4 --output-format csv -- \
  python3 bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/mem.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o c4 --output-format csv -- \
  python3 bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/fetch.log 2>&1 || exit 1
echo done
