# final check B (profiles, C4 and C5 lines) followed by the stage-1 partitions-in-flight probe
bash tools/r03_final3B.sh || exit 1
mkdir -p gpurun_out/probe
timeout -k 10 300 python -u tools/dual_mst_probe.py 2 10 > gpurun_out/probe/dual.json 2>&1 || { echo "probe failed"; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --mst-workers 2 > gpurun_out/probe/c2_w2.json.log 2>&1 || { echo "w2 failed"; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --mst-workers 3 > gpurun_out/probe/c2_w3.json.log 2>&1 || { echo "w3 failed"; exit 1; }
echo done
