#!/bin/bash
# rows-path thresholds, second pass (C2 A/B)
set -o pipefail
mkdir -p gpurun_out/r04u
AB_REPS=3 bash tools/ab_c2.sh rm4 krm8 > gpurun_out/r04u/ab_c2.log 2>&1
echo done
