# round-3 final (A): full GPU suite, smoke, C2 bench (with CPU baseline), C3 line
OUT=gpurun_out/finalA; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python -u bench.py > $OUT/bench_c2.json.log 2>&1 || { echo "bench failed"; exit 1; }
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline > $OUT/bench_c3.json.log 2>&1 || { echo "c3 failed"; exit 1; }
echo done
