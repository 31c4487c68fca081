# C2 step pipeline: bench N=1 (twice), a 2-rank gloo rehearsal of the N>1 path on the one device
mkdir -p gpurun_out/pipe && export TMPDIR=/tmp && \
timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/pipe/c2_n1a.json.log 2>&1 && \
timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/pipe/c2_n1b.json.log 2>&1 && \
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > gpurun_out/pipe/c2_n2_gloo.json.log 2>&1; echo rc=$?
