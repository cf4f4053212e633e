#!/bin/bash
# Round 6: attention parity tests on a build_variants library, then a same-box A/B against another (kernel_bench
# attention). Usage (GPU box): bash tools/r6_variant_ab.sh <tag> <tested variant> "<variants>" [rounds]
TAG=$1; TV=$2; VARS=$3; R=${4:-3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
LCI_LIB_PATH=$ROOT/build_variants/liblci_$TV.so timeout -k 10 600 python -u -m pytest $ROOT/tests/test_attention_gpu.py \
  $ROOT/tests/test_attention_long_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/gputest_$TV.log 2>&1
rc=$?; tail -3 $OUT/gputest_$TV.log; [ $rc -eq 0 ] || { echo "STOP tests rc $rc"; exit 1; }
bash $ROOT/tools/lib_ab.sh $TAG "$VARS" $R python $ROOT/tools/kernel_bench.py attention
