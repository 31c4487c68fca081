# merge of presorted runs: parity tests, microbench, bench N=1 and a 2-rank gloo rehearsal of the N>1 C2 step
mkdir -p gpurun_out/merge && export TMPDIR=/tmp && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "merge_sorted or sort_edges or sharded or gather or merge_edges" tests/test_gpu_sharded.py > gpurun_out/merge/tests.log 2>&1 && \
timeout -k 10 120 python -u tools/merge_bench.py 8 1999999 10 > gpurun_out/merge/mb.log 2>&1 && \
timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/merge/c2_n1.json.log 2>&1 && \
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > gpurun_out/merge/c2_n2_gloo.json.log 2>&1; echo rc=$?
