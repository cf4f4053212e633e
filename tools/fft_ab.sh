# FFT conv A/B on one box: the Hyena tests, kernel_bench fftconv, and a kernel trace of it.
mkdir -p gpurun_out/r02h
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hyena_gpu.py > gpurun_out/r02h/t5.log 2>&1 || { tail -30 gpurun_out/r02h/t5.log; exit 1; }
tail -1 gpurun_out/r02h/t5.log
LCI_NO_KTIMER=1 timeout -k 10 120 python -u tools/kernel_bench.py fftconv > gpurun_out/r02h/fft5.txt 2>&1 || exit 1
cut -c1-120 gpurun_out/r02h/fft5.txt
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02h/fftprof -o run -- python3 $GRAFT_REPO_ROOT/tools/kernel_bench.py fftconv > $GRAFT_REPO_ROOT/gpurun_out/r02h/fftprof.log 2>&1
