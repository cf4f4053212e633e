#!/bin/bash
# Linear weight-gradient split granularity A/B on the C3 step (graph mode) and the metric step: the default rule
# (partial-traffic capped, down to 512 rows per split) vs the former fixed 2048-row minimum (LCI_LW_MINROWS=2048).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/lwab3
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_linear_gpu.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/test.log 2>&1; rc=$?; tail -1 $OUT/test.log; [ $rc -eq 0 ] || exit $rc
for w in swin_p2_128 vit_p2_512; do
  for v in 0 2048 0 2048; do
    LCI_LW_MINROWS=$v timeout -k 10 300 python -u bench.py --workload $w --steps 6 --warmup 2 --no-cpu-baseline \
      --no-secondary > $OUT/b_${w}_$v.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/b_${w}_$v.json'));k=d['kernels'];print('$w', $v, d['ms_per_step'], k['linear_wgrad']['ms_per_step'])" | tee -a $OUT/summary.txt
  done
done
