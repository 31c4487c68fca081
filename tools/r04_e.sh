#!/bin/bash
# round 4 check E: K2b late-round publish / refresh A/B
set -uo pipefail
OUT=gpurun_out/r04e; mkdir -p $OUT; export TMPDIR=/tmp
AB_REPS=2 timeout -k 10 1000 bash tools/ab_c2.sh nodpp pubw refr5 refr2 > $OUT/ab_c2.log 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_c2.log; exit 1; }
echo done
