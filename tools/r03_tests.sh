# full GPU test suite + smoke + default bench (C2) into $1
OUT=${1:?outdir}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gputest.log" 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 200 python bench.py > "$OUT/bench_c2.json.log" 2>&1 || { echo "bench failed"; exit 1; }
echo done
