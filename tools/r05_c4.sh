#!/bin/bash
# C4: MFMA tests, A/B of the LDS-staged screen log + XCD-contiguous re-check, PMC passes of the default
set -uo pipefail
OUT=$(readlink -f "${1:?outdir}")
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py -x -v --timeout 600 --timeout-method thread > "$OUT/t_mfma.log" 2>&1 || { echo "mfma tests failed"; tail -30 "$OUT/t_mfma.log"; exit 1; }
AB_REPS=2 timeout -k 10 900 bash tools/ab_c4.sh k1old k1lb > "$OUT/ab.log" 2>&1 || { echo "ab failed"; cat "$OUT/ab.log"; exit 1; }
timeout -k 10 500 bash tools/profile_c4.sh "$OUT/pmc" > "$OUT/pmc.log" 2>&1 || { echo "pmc failed"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/pmc/pmc_summary.json'))
for k,v in d.items():
  if 'screen' in k or 'final16' in k: print(k, round(v['hbm_read_bytes_per_launch']/1e9,2), round(v['hbm_write_bytes_per_launch']/1e9,2))"
cat "$OUT/ab.log"
