#!/bin/bash
# C4: permlane probe, MFMA tests, A/B (ab/k1old = round-4 screen/re-check code), PMC passes of the default
set -uo pipefail
OUT=$(readlink -f "${1:?outdir}")
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 60 ./ab/probe/permlane_probe > "$OUT/probe.log" 2>&1 || { echo "probe failed"; cat "$OUT/probe.log"; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py -x -v --timeout 600 --timeout-method thread > "$OUT/t_mfma.log" 2>&1 || { echo "mfma tests failed"; tail -30 "$OUT/t_mfma.log"; exit 1; }
AB_REPS=2 timeout -k 10 900 bash tools/ab_c4.sh ${AB_VARIANTS:-k1old} > "$OUT/ab.log" 2>&1 || { echo "ab failed"; cat "$OUT/ab.log"; exit 1; }
[ -n "${SKIP_PMC:-}" ] || { timeout -k 10 500 bash tools/profile_c4.sh "$OUT/pmc" > "$OUT/pmc.log" 2>&1 || { echo "pmc failed"; exit 1; }; }
[ -n "${SKIP_PMC:-}" ] || python3 -c "
import json; d=json.load(open('$OUT/pmc/pmc_summary.json'))
for k,v in d.items():
  if 'screen' in k or 'final16' in k: print(k, round(v['hbm_read_bytes_per_launch']/1e9,2), round(v['hbm_write_bytes_per_launch']/1e9,2))"
cat "$OUT/probe.log" "$OUT/ab.log"; grep -c PASSED "$OUT/t_mfma.log"
