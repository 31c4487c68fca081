# bench value from HBM-resident inputs: C2 (N=1 and a 2-rank gloo rehearsal on one GPU) and C4
OUT=gpurun_out/benchsem; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/c2.json.log 2>&1 || { echo "c2 failed"; exit 1; }
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --no-cpu-baseline > $OUT/c2_n2_gloo.json.log 2>&1 || { echo "c2 n2 failed"; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline > $OUT/c4.json.log 2>&1 || { echo "c4 failed"; exit 1; }
echo done
