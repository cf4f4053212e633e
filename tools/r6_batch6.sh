#!/bin/bash
# Round 6: split-sum kernels -- parity, then the metric and C3 steps with LCI_HIP_SPLITSUM 0 / 1 alternating.
# Usage (GPU box): bash tools/r6_batch6.sh <tag>
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  $ROOT/tests/test_sum_splits_gpu.py $ROOT/tests/test_conv_gpu.py $ROOT/tests/test_modules_gpu.py $ROOT/tests/test_gemm_gpu.py \
  > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "STOP tests rc $rc"; exit 1; }
for ss in 0 1 0 1; do
  LCI_HIP_SPLITSUM=$ss timeout -k 10 400 python -u $ROOT/bench.py --no-cpu-baseline --no-secondary --steps 6 --warmup 2 \
    > $OUT/m_ss$ss.json 2>> $OUT/m.err || { echo "STOP metric ss$ss"; tail -5 $OUT/m.err; exit 1; }
  echo "metric splitsum=$ss $(python3 -c "import json;d=json.loads(open('$OUT/m_ss$ss.json').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
  LCI_HIP_SPLITSUM=$ss timeout -k 10 300 python -u $ROOT/bench.py --workload swin_p2_128 --steps 10 --warmup 3 --no-cpu-baseline \
    > $OUT/c3_ss$ss.json 2>> $OUT/c3.err || { echo "STOP c3 ss$ss"; tail -5 $OUT/c3.err; exit 1; }
  echo "c3 splitsum=$ss $(python3 -c "import json;d=json.loads(open('$OUT/c3_ss$ss.json').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
done
echo "batch6 $TAG done"
