# final check D: the default C2 line (partitions in flight) with its CPU baseline, its rocprofv3
# stats + PMC passes, and a 2-rank gloo rehearsal of the default pipeline on one GPU
OUT=gpurun_out/final3d; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > $OUT/bench_c2.json.log 2>&1 || { echo "bench failed"; exit 1; }
timeout -k 10 600 bash tools/profile_bench.sh $OUT/prof_c2 > $OUT/prof_c2.log 2>&1 || { echo "profile failed"; exit 1; }
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 2 --backend gloo --no-cpu-baseline > $OUT/c2_n2_gloo.json.log 2>&1 || { echo "n2 failed"; exit 1; }
echo done
