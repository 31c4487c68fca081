#!/bin/bash
# K1m re-check from a layout-order FP64 copy: MFMA parity tests, then the C4 A/B
set -o pipefail
mkdir -p gpurun_out/${R04M_OUT:-r04m}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${R04M_OUT:-r04m}/tests.log 2>&1 || { echo tests failed; exit 1; }
AB_REPS=2 bash tools/ab_c4.sh ${AB_VARIANTS:-xlay0} > gpurun_out/${R04M_OUT:-r04m}/ab_c4.log 2>&1
echo done
