mkdir -p gpurun_out/r02h
for pb in 4 2 6 8 12; do
  echo "pb $pb" >> gpurun_out/r02h/fftpb.txt
  LCI_FFT_ROW_PB=$pb LCI_NO_KTIMER=1 timeout -k 10 120 python -u tools/kernel_bench.py fftconv >> gpurun_out/r02h/fftpb.txt 2>&1 || exit 1
done
LCI_FFT_ROW_PB=6 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hyena_gpu.py > gpurun_out/r02h/t6.log 2>&1; tail -1 gpurun_out/r02h/t6.log
grep -v amdgpu.ids gpurun_out/r02h/fftpb.txt | cut -c1-100
