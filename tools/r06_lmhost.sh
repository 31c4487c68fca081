#!/bin/bash
# host local-model changes: every GPU test that runs local models (parity vs the oracle, scaled
# C5 fixtures, sharded driver, C1, model pool threads), then the one-model bench
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mr_scaled.py tests/test_gpu_sharded.py tests/test_gpu_c1.py tests/test_gpu_driver.py tests/test_gpu_threads.py -x -q --timeout 300 --timeout-method thread > "$OUT/t.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/t.log"; exit 1; }
tail -1 "$OUT/t.log"
timeout -k 10 300 python -u tools/lm_bench.py 16384 8 3 > "$OUT/lm.log" 2>&1 || { echo "lm bench failed"; tail "$OUT/lm.log"; exit 1; }
cat "$OUT/lm.log" | grep "^{"
