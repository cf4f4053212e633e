#!/bin/bash
# Selective-scan A/B on the GPU box: parity tests under the first variant, then kernel_bench scan at L=65536 / 2^21
# for each variant (alternating, twice). A variant is a space-free env assignment list joined by commas, e.g.
#   bash tools/scan_ab.sh tag LCI_SCAN_BWD_WAVES=1 LCI_SCAN_BWD_WAVES=4 LCI_SCAN_PF=0,LCI_SCAN_WAVES=16384
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${1:-scan_ab}; shift
mkdir -p $OUT
first=${1:-LCI_SCAN_PF=1}
env ${first//,/ } timeout -k 10 300 python -u -m pytest tests/test_mamba_gpu.py tests/test_scan_long_gpu.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2; do
  for v in "$@"; do
    echo "$v run $r" | tee -a $OUT/ab.txt
    env ${v//,/ } timeout -k 10 120 python -u tools/kernel_bench.py scan >> $OUT/ab.txt 2>&1 || exit 1
  done
done
grep -E "run [12]|selective" $OUT/ab.txt | sed 's/, "achieved.*//'
