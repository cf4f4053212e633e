#!/bin/bash
# Round 6: the full GPU suite on the tree, then the C3 step with the window-attention workgroup order 0 / 1
# (alternating, same box) and the metric bench line.
# Usage (GPU box): bash tools/r6_batch5.sh <tag>
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $ROOT/tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "STOP tests rc $rc"; exit 1; }
for wo in 0 1 0 1 0 1; do
  LCI_WIN_ORDER=$wo timeout -k 10 300 python -u $ROOT/bench.py --workload swin_p2_128 --steps 10 --warmup 3 --no-cpu-baseline \
    > $OUT/c3_o$wo.json 2>> $OUT/c3.err || { echo "STOP c3 o$wo"; tail -5 $OUT/c3.err; exit 1; }
  echo "win_order=$wo $(python3 -c "import json;d=json.loads(open('$OUT/c3_o$wo.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['kernels'].get('window_attn_bwd'), d['kernels'].get('window_attn_fwd'))")"
done
timeout -k 10 600 python -u $ROOT/bench.py > $OUT/metric.json 2> $OUT/metric.err || { echo "STOP metric"; tail -5 $OUT/metric.err; exit 1; }
cut -c1-300 $OUT/metric.json
echo "batch5 $TAG done"
