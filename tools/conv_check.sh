#!/bin/bash
# Conv GPU tests + per-shape conv bench (C3 set and two C5 shapes). Usage (GPU box): bash tools/conv_check.sh <tag>
TAG=${1:-conv}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $ROOT/tests/test_conv_gpu.py $ROOT/tests/test_upernet.py $ROOT/tests/test_linear_gpu.py -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
rc=$?; tail -2 $OUT/gputest.log; [ $rc -le 1 ] || { echo "STOP tests rc $rc"; exit $rc; }
timeout -k 10 400 python -u $ROOT/tools/conv_bench.py --set c3 --passes fwd,dgrad > $OUT/conv_c3.jsonl 2>&1 || exit 1
for o in 256-256 128-64; do
  timeout -k 10 300 python -u $ROOT/tools/conv_bench.py --set c5 --only $o --passes fwd,dgrad >> $OUT/conv_c5.jsonl 2>&1 || exit 1
done
echo "conv_check $TAG done"
