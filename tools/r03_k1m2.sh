# K1m register top lists: MFMA parity tests, the cycle split (profiling build), C4 A/B
OUT=gpurun_out/k1m2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread > $OUT/mfma_tests.log 2>&1 || { echo "mfma tests failed"; exit 1; }
HDBMI_LIB=$PWD/ab/k1_prof/libhdbmi.so K1M_QUICK=1 K1M_PROF=1 K1M_DIAG=1 timeout -k 10 200 python -u tools/k1m_bench.py 2000000 128 > $OUT/k1m_prof.json 2>&1 || { echo "k1m prof failed"; exit 1; }
timeout -k 10 600 bash tools/ab_c4.sh "$@" > $OUT/ab.log 2>&1 || { echo "ab failed"; exit 1; }
echo done
