#!/bin/bash
# FFT plan sweep (runtime knobs LCI_FFT_LN1 / LCI_FFT_G): bash tools/fft_sweep.sh
for cfg in "8 8" "8 16" "7 16" "8 4"; do set -- $cfg
  echo "== LN1=$1 G=$2"
  LCI_FFT_LN1=$1 LCI_FFT_G=$2 timeout -k 10 120 python tools/kernel_bench.py fftconv 2>&1 | grep kernel
done
