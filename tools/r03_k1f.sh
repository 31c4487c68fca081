# re-check with 16 lanes per query (variant build ab/k1f_qpw4): MFMA parity tests on it, then C4 A/B
OUT=gpurun_out/k1f2; mkdir -p $OUT; export TMPDIR=/tmp
HDBMI_LIB=$PWD/ab/k1f_qpw4/libhdbmi.so timeout -k 10 400 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread > $OUT/mfma_tests.log 2>&1 || { echo "mfma tests failed"; exit 1; }
timeout -k 10 600 bash tools/ab_c4.sh k1f_qpw4 > $OUT/ab.log 2>&1 || { echo "ab failed"; exit 1; }
echo done
