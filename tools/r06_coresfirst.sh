#!/bin/bash
# cores-first local models: equality test, driver / C5-fixture tests, then the C5 line (with its
# rank emulation) with HDB_CORES_FIRST=1 and 0
mkdir -p gpurun_out
set -uo pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_local_model_cores.py tests/test_gpu_mr_scaled.py tests/test_gpu_sharded.py tests/test_gpu_c1.py tests/test_gpu_driver.py tests/test_gpu_threads.py -x -q --timeout 300 --timeout-method thread > "$OUT/t.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/t.log"; exit 1; }
tail -1 "$OUT/t.log"
for x in 1 0; do
  HDB_CORES_FIRST=$x HDB_NATIVE_BACKTRACE=1 timeout -k 10 600 python -u bench.py --workload c5 --phases --no-cpu-baseline > "$OUT/c5_$x.json.log" 2> "$OUT/c5_$x.err" || { echo "c5 $x failed"; tail "$OUT/c5_$x.err"; exit 1; }
  tail -1 "$OUT/c5_$x.json.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['predicted_scaling']; print('cores_first=$x', round(d['ms_per_step']), 'ms', p['speedup'], {k: round(v['local_models'], 3) for k, v in p['phases'].items()})"
done
