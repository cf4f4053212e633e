#!/bin/bash
# Same-box A/B of the selective scan between this tree and a second built tree in tmp_ab/ (git worktree of an
# earlier commit, built on the CPU side): scan parity tests on this tree, then kernel_bench scan alternating.
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${AB_TAG:-scan_ab6}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_mamba_gpu.py tests/test_scan_long_gpu.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  echo "old run $r" >> $OUT/ab.txt; (cd tmp_ab && timeout -k 10 120 python -u tools/kernel_bench.py scan) >> $OUT/ab.txt 2>&1 || exit 1
  echo "new run $r" >> $OUT/ab.txt; timeout -k 10 120 python -u tools/kernel_bench.py scan >> $OUT/ab.txt 2>&1 || exit 1
done
grep -E "run [12]|selective_scan_bwd" $OUT/ab.txt | sed 's/, "achieved.*//'
