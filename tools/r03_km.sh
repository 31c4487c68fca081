# MFMA k-means layout: MFMA parity tests, C4 A/B (VALU assignment variant), then the bench lines
# from HBM-resident inputs (C2 N=1, a 2-rank gloo rehearsal on one GPU, C4)
OUT=gpurun_out/km; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread > $OUT/mfma_tests.log 2>&1 || { echo "mfma tests failed"; exit 1; }
timeout -k 10 600 bash tools/ab_c4.sh k1_kmvalu > $OUT/ab.log 2>&1 || { echo "ab failed"; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/c2.json.log 2>&1 || { echo "c2 failed"; exit 1; }
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --no-cpu-baseline > $OUT/c2_n2_gloo.json.log 2>&1 || { echo "c2 n2 failed"; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline > $OUT/c4.json.log 2>&1 || { echo "c4 failed"; exit 1; }
echo done
