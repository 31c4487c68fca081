# round-3 final (session 3, A): full GPU suite, smoke, C2 line (with the CPU baseline), C3 line
OUT=gpurun_out/final3; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python -u bench.py > $OUT/bench_c2.json.log 2>&1 || { echo "bench failed"; exit 1; }
timeout -k 10 300 python -u bench.py --workload c3 > $OUT/bench_c3.json.log 2>&1 || { echo "c3 failed"; exit 1; }
echo done
