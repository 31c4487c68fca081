# K1m screen: MFMA parity tests on the in-tree build, then C4 A/B against variant builds under ab/
OUT=gpurun_out/k1m; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread > $OUT/mfma_tests.log 2>&1 || { echo "mfma tests failed"; exit 1; }
timeout -k 10 600 bash tools/ab_c4.sh "$@" > $OUT/ab.log 2>&1 || { echo "ab failed"; exit 1; }
echo done
