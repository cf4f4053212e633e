#!/bin/bash
# Round-4 attention A/B: parity suite on the default build, then old / new liblci variants alternating.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r4attn}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest $ROOT/tests/test_attention_gpu.py $ROOT/tests/test_attention_long_gpu.py -m gpu -x -v \
  --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || { echo "STOP tests rc $rc"; exit 1; }
bash $ROOT/tools/lib_ab.sh ${1:-r4attn} "${2:-old new}" ${3:-2} python $ROOT/tools/kernel_bench.py attention
grep -h "attn_bwd_dkdv\|attn_bwd_dq\|==" $OUT/ab.txt | sed "s/\"achieved.*//"
