# round-3 final (session 3, B): C2 profile (kernel stats + PMC passes), C4 stats + PMC passes,
# then the C4 line (reading the fresh PMC summary) and the C5 line with phases
OUT=gpurun_out/final3; mkdir -p $OUT/c4_final; export TMPDIR=/tmp
timeout -k 10 600 bash tools/profile_bench.sh $OUT/prof_c2 > $OUT/prof_c2.log 2>&1 || { echo "profile c2 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c4_final/stats -o c4 --output-format csv -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c4_final/bench_c4.json.log 2> $OUT/c4_stats.err || { echo "c4 stats failed"; exit 1; }
timeout -k 10 500 bash tools/profile_c4.sh $OUT/c4_final > $OUT/prof_c4.log 2>&1 || { echo "profile c4 failed"; exit 1; }
mkdir -p profiles/r03/c4_final profiles/r03/final/prof_c2 && cp $OUT/c4_final/pmc_summary.json profiles/r03/c4_final/ && cp $OUT/prof_c2/pmc_summary.json profiles/r03/final/prof_c2/
timeout -k 10 300 python -u bench.py --workload c4 > $OUT/bench_c4.json.log 2>&1 || { echo "c4 failed"; exit 1; }
timeout -k 10 300 python -u bench.py --workload c5 --phases > $OUT/bench_c5.json.log 2>&1 || { echo "c5 failed"; exit 1; }
echo done
