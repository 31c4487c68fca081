#!/bin/bash
# round 4 check G: K1t row-batched leaf groups -- parity (tree + parity tests), C2 A/B
set -uo pipefail
OUT=gpurun_out/r04g; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py tests/test_gpu_c1.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
AB_REPS=2 timeout -k 10 900 bash tools/ab_c2.sh k1trows0 nodpp pubw refr5 > $OUT/ab_c2.log 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_c2.log; exit 1; }
echo done
