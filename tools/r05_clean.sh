#!/bin/bash
mkdir -p gpurun_out  # every run keeps its stderr (tools_stderr.log)
# after the knob cleanup: tree / mfma / parity / c1 tests, then the C2 and C4 lines
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_mfma.py tests/test_gpu_parity.py tests/test_gpu_c1.py -x -q --timeout 300 --timeout-method thread > "$OUT/t.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/t.log"; exit 1; }
tail -1 "$OUT/t.log"
timeout -k 10 300 python -u bench.py --steps 40 --no-cpu-baseline > "$OUT/c2.json.log" 2>>gpurun_out/tools_stderr.log || { echo c2 failed; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline > "$OUT/c4.json.log" 2>>gpurun_out/tools_stderr.log || { echo c4 failed; exit 1; }
for f in c2 c4; do tail -1 "$OUT/$f.json.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value']/1e6,2), round(d['ms_per_step'],3))"; done
