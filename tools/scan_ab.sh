#!/bin/bash
# Selective-scan A/B on the GPU box: parity tests with the default build, then kernel_bench scan at L=65536 / 2^21
# for the forward load pipelining (LCI_SCAN_PF) x the chunk-count target (LCI_SCAN_WAVES).
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${1:-scan_ab}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_mamba_gpu.py tests/test_scan_long_gpu.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for pf in 0 1; do
  for w in ${WAVES:-8192 16384 24576}; do
    echo "PF=$pf WAVES=$w" | tee -a $OUT/ab.txt
    LCI_SCAN_PF=$pf LCI_SCAN_WAVES=$w timeout -k 10 120 python -u tools/kernel_bench.py scan >> $OUT/ab.txt 2>&1 || exit 1
  done
done
grep -E "PF=|selective" $OUT/ab.txt | sed 's/"work_per_launch.*//'
