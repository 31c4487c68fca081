# round-3 final (B): C2 profile (kernel stats + PMC passes), C5 line with phases, C4 line
OUT=gpurun_out/finalB; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 bash tools/profile_bench.sh $OUT/prof_c2 > $OUT/prof_c2.log 2>&1 || { echo "profile failed"; exit 1; }
timeout -k 10 300 python -u bench.py --workload c5 --phases > $OUT/bench_c5.json.log 2>&1 || { echo "c5 failed"; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4 > $OUT/bench_c4.json.log 2>&1 || { echo "c4 failed"; exit 1; }
echo done
