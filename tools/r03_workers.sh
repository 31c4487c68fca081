# C2 with several partitions in flight: stage-1 workers x label stages, plus a 2-rank gloo rehearsal
OUT=gpurun_out/workers; mkdir -p $OUT; export TMPDIR=/tmp
for c in "1 1" "2 2" "3 3" "2 3" "3 2"; do set -- $c
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --mst-workers $1 --label-workers $2 > $OUT/c2_m$1_l$2.json.log 2>&1 || { echo "m$1 l$2 failed"; exit 1; }
done
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 2 --backend gloo --no-cpu-baseline --mst-workers 2 > $OUT/c2_n2_gloo_m2.json.log 2>&1 || { echo "n2 failed"; exit 1; }
echo done
