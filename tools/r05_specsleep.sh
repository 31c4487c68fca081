#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# speculative Prim (slots 6) in the C5 job with sleeping worker waits (ab/sp2, ab/sp8)
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in sp2 sp8; do
  HDBMI_LIB=$PWD/ab/$v/libhdbmi.so HDB_PRIM_COOP_SLOTS=6 timeout -k 10 300 python -u bench.py --workload c5 --phases --no-cpu-baseline > "$OUT/c5_$v.json.log" 2>>gpurun_out/tools_stderr.log || { echo c5 failed; exit 1; }
  tail -1 "$OUT/c5_$v.json.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', round(d['ms_per_step'],1), r.get('us_per_step'), d['local_model_s']['core'], d['local_model_s']['prim'], d.get('prim_coop_plain_retries'))"
done
