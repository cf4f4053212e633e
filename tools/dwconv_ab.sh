#!/bin/bash
# Mamba dwconv + SiLU on the GPU box: mamba parity tests, kernel_bench dwconv with the vector paths on / off,
# then (optional, $1 = c5) the C5 bench line.
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${DW_TAG:-dw_ab3}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_mamba_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in "LCI_DWCONV_BWD_V=4" "LCI_DWCONV_BWD_V=0" "LCI_DWCONV_BWD_V=8" "LCI_DWCONV_VEC=0"; do
  echo "$v" >> $OUT/ab.txt
  env $v timeout -k 10 120 python -u tools/kernel_bench.py dwconv >> $OUT/ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/ab.txt | sed 's/, "work_per_launch.*//'
if [ "$1" = c5 ]; then
  timeout -k 10 600 python -u bench.py --workload vit_mamba_p2_256 --steps 3 --warmup 2 --no-cpu-baseline \
    > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit 1
  cut -c1-260 $OUT/bench_c5.json
fi
