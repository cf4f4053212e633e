#!/bin/bash
# Round 6: Adam kernel with 4096-element workgroups (16 loads in flight per thread, bias corrections once per
# workgroup) -- optimizer / C1 train-step parity on the tree's library, then a same-box A/B of build_variants
# liblci_adamnew (the tree) and liblci_adamold (HEAD's optim.hip) on tools/adam_bench.py.
# Usage (GPU box): bash tools/r6_adam_ab.sh <tag>
TAG=${1:-r6ad}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $ROOT/tests/test_optim_gpu.py $ROOT/tests/test_c1_train_step_gpu.py $ROOT/tests/test_graph_gpu.py \
  -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || { echo "STOP tests rc $rc"; exit 1; }
cd $ROOT && bash $ROOT/tools/lib_ab.sh $TAG "adamold adamnew" 3 python $ROOT/tools/adam_bench.py
