#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/attab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $ROOT/tests/test_attention_gpu.py $ROOT/tests/test_attention_long_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
rc=$?; tail -2 $OUT/gputest.log; [ $rc -eq 0 ] || { echo "STOP tests rc $rc"; exit 1; }
bash $ROOT/tools/lib_ab.sh attab "old new" 3 python $ROOT/tools/kernel_bench.py attention
