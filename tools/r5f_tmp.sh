export TMPDIR=/tmp
OUT=gpurun_out/r5f
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_hyena_gpu.py tests/test_hyena_filter_gpu.py tests/test_swin_alt_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/test.log 2>&1 || { echo "STOP test"; tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
timeout -k 10 300 python -u tools/kernel_bench.py fftconv > $OUT/kb.jsonl 2> $OUT/kb.err || { echo "STOP kb"; tail $OUT/kb.err; exit 1; }
cat $OUT/kb.jsonl
