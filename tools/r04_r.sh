#!/bin/bash
# K3g union-box runs: nearest-sample parity tests, then the C5 A/B
set -o pipefail
mkdir -p gpurun_out/r04r
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k nearest -x -q --timeout 200 --timeout-method thread > gpurun_out/r04r/tests.log 2>&1 || { echo tests failed; exit 1; }
AB_REPS=2 bash tools/ab_c5.sh sb0 sb4 sb16 > gpurun_out/r04r/ab_c5.log 2>&1
echo done
