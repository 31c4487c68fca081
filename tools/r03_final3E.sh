# final check E (after the K1m WPE change): full GPU suite, smoke, C4 stats + PMC passes, C4 line
OUT=gpurun_out/final3e; mkdir -p $OUT/c4_final; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c4_final/stats -o c4 --output-format csv -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c4_final/bench_c4.json.log 2> $OUT/c4_stats.err || { echo "c4 stats failed"; exit 1; }
timeout -k 10 500 bash tools/profile_c4.sh $OUT/c4_final > $OUT/prof_c4.log 2>&1 || { echo "profile c4 failed"; exit 1; }
cp $OUT/c4_final/pmc_summary.json profiles/r03/c4_final/
timeout -k 10 300 python -u bench.py --workload c4 > $OUT/bench_c4.json.log 2>&1 || { echo "c4 failed"; exit 1; }
echo done
