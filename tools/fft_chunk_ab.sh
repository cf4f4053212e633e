mkdir -p gpurun_out/r02h
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hyena_gpu.py > gpurun_out/r02h/t4.log 2>&1 || { tail -20 gpurun_out/r02h/t4.log; exit 1; }
LCI_FFT_CHUNK_MB=16 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hyena_gpu.py >> gpurun_out/r02h/t4.log 2>&1 || { tail -20 gpurun_out/r02h/t4.log; exit 1; }
tail -1 gpurun_out/r02h/t4.log
for mb in 0 32 64 128 256; do
  echo "chunk $mb" >> gpurun_out/r02h/fftab.txt
  LCI_FFT_CHUNK_MB=$mb LCI_NO_KTIMER=1 timeout -k 10 120 python -u tools/kernel_bench.py fftconv >> gpurun_out/r02h/fftab.txt 2>&1 || exit 1
done
cat gpurun_out/r02h/fftab.txt | cut -c1-200
