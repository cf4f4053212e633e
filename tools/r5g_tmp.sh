export TMPDIR=/tmp
OUT=gpurun_out/r5g
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_scan_long_gpu.py -m gpu -q -s --timeout 300 --timeout-method thread > $OUT/scan_test.log 2>&1 || { echo "STOP scantest"; tail -20 $OUT/scan_test.log; exit 1; }
grep "L=" $OUT/scan_test.log; tail -1 $OUT/scan_test.log
bash tools/pmc_r5.sh pmc_r5 attention scan gemm || exit 1
