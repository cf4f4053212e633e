# A/B of the wide column pass workgroup size (complex elements per workgroup) on kernel_bench fftconv.
mkdir -p gpurun_out/r02h
rm -f gpurun_out/r02h/fftcw.txt
for cw in 8192 4096; do
  echo "cw $cw" >> gpurun_out/r02h/fftcw.txt
  LCI_FFT_CW=$cw LCI_NO_KTIMER=1 timeout -k 10 120 python -u tools/kernel_bench.py fftconv >> gpurun_out/r02h/fftcw.txt 2>&1 || exit 1
done
LCI_FFT_CW=4096 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hyena_gpu.py > gpurun_out/r02h/t8.log 2>&1; tail -1 gpurun_out/r02h/t8.log
grep -v amdgpu.ids gpurun_out/r02h/fftcw.txt | cut -c1-100
