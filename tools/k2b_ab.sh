# K2b A/B: variant build under ab/<v>: exact-MST GPU tests with it, per-round stats, then C2 pairs
V=${1:?variant}
mkdir -p gpurun_out/k2b_ab && export TMPDIR=/tmp && \
HDBMI_LIB=$PWD/ab/$V/libhdbmi.so timeout -k 10 400 python -u -m pytest tests/test_gpu_tree.py -x -q --timeout 300 --timeout-method thread > gpurun_out/k2b_ab/test_$V.log 2>&1 && \
HDBMI_LIB=$PWD/ab/$V/libhdbmi.so timeout -k 10 200 python -u tools/boruvka_stats.py > gpurun_out/k2b_ab/stats_$V.log 2>&1 && \
bash tools/ab_c2.sh $V > gpurun_out/k2b_ab/ab_$V.log 2>&1; echo rc=$?
