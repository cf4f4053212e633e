#!/bin/bash
# Round 6: attention parity tests on the tree's library, then a same-box A/B of build_variants (kernel_bench attention).
# Usage (GPU box): bash tools/r6_attn_ab.sh <tag> "<variants>" [rounds]
TAG=$1; VARS=$2; R=${3:-3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $ROOT/tests/test_attention_gpu.py $ROOT/tests/test_attention_long_gpu.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || { echo "STOP tests rc $rc"; exit 1; }
bash $ROOT/tools/lib_ab.sh $TAG "$VARS" $R python $ROOT/tools/kernel_bench.py attention
