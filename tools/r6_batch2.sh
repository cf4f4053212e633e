#!/bin/bash
# Round 6: the changed parity tests on the tree's library, then a same-box attention A/B of build_variants.
# Usage (GPU box): bash tools/r6_batch2.sh <tag> "<variants>" <rounds>
TAG=$1; VARS=$2; R=${3:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PYT="python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 1000 $PYT $ROOT/tests/test_attention_gpu.py $ROOT/tests/test_attention_long_gpu.py $ROOT/tests/test_mamba_gpu.py \
  $ROOT/tests/test_optim_gpu.py $ROOT/tests/test_modules_gpu.py $ROOT/tests/test_ddp_model_gpu.py $ROOT/tests/test_scan_long_gpu.py \
  $ROOT/tests/test_swin_alt_gpu.py $ROOT/tests/test_c1_train_step_gpu.py $ROOT/tests/test_ddp.py > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "STOP tests rc $rc"; exit 1; }
[ -n "$VARS" ] && { bash $ROOT/tools/lib_ab.sh $TAG "$VARS" $R python $ROOT/tools/kernel_bench.py attention || exit 1; }
echo "batch2 $TAG done"
