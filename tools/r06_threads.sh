#!/bin/bash
# the model pool under 8 threads / 12 hardware queues, stderr kept.
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
export HDB_NATIVE_BACKTRACE=1
HDB_HW_QUEUES=12 timeout -k 10 300 python -u -X faulthandler tools/thread_stress.py --threads 8 --rounds 2 \
    > "$OUT/stress.log" 2> "$OUT/stress.err" || { echo "stress failed rc=$?"; exit 1; }
tail -3 "$OUT/stress.log"
HDB_MODEL_THREADS=8 HDB_HW_QUEUES=12 timeout -k 10 400 python -u -X faulthandler bench.py --workload c5 --phases \
    --no-cpu-baseline > "$OUT/c5_t8_q12.json.log" 2> "$OUT/c5_t8_q12.err" || { echo "c5 failed rc=$?"; exit 1; }
tail -1 "$OUT/c5_t8_q12.json.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 t8 q12', round(d['ms_per_step'],1), 'ms', d['predicted_scaling']['speedup'])"
