#!/bin/bash
# Round 6: conv weight gradient v6 (LDS-DMA staging) -- conv / UNETR / UperNet / module parity on the tree's library,
# then same-box A/B of LCI_WGRAD_DMA=1 (v6) against 0 (v5): conv_bench C3 weight gradients and the C3 bench line.
# Usage (GPU box): bash tools/r6_wgrad_ab.sh <tag>
TAG=${1:-r6wg}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $ROOT/tests/test_conv_gpu.py $ROOT/tests/test_unetr.py $ROOT/tests/test_upernet.py \
  $ROOT/tests/test_modules_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || { echo "STOP tests rc $rc"; exit 1; }
for r in 1 2; do
  for v in 0 1; do
    echo "== LCI_WGRAD_DMA=$v round $r" >> $OUT/conv_ab.txt
    LCI_WGRAD_DMA=$v timeout -k 10 300 python $ROOT/tools/conv_bench.py --set c3 --passes wgrad >> $OUT/conv_ab.txt 2>&1 || { echo "STOP conv $v"; exit 1; }
    LCI_WGRAD_DMA=$v timeout -k 10 300 python $ROOT/tools/conv_bench.py --set 2d --passes wgrad >> $OUT/conv_ab.txt 2>&1 || { echo "STOP conv2d $v"; exit 1; }
  done
done
for v in 0 1 0 1; do
  LCI_WGRAD_DMA=$v timeout -k 10 400 python $ROOT/bench.py --workload swin_p2_128 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c3_$v.json 2> $OUT/c3_$v.err \
    || { echo "STOP bench $v"; tail -3 $OUT/c3_$v.err; exit 1; }
  python3 -c "import json,sys; j=json.loads(open('$OUT/c3_$v.json').read().strip().splitlines()[-1]); print('C3 LCI_WGRAD_DMA=$v', j['ms_per_step'], j['kernels'].get('conv3_wgrad'))" | tee -a $OUT/c3_ab.txt
done
echo "r6_wgrad_ab $TAG done"
