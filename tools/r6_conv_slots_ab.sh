#!/bin/bash
# Round 6: three-slot LDS-DMA conv forward -- conv / UNETR / UperNet / module parity on the tree's library, then a
# same-box A/B of build_variants liblci_slots3 (the tree) and liblci_slots2 (-DLCI_CONV_FWD_SLOTS=2): conv_bench C3 / C5
# / 2-D forward and data gradient, and the C3 bench line. Usage (GPU box): bash tools/r6_conv_slots_ab.sh <tag>
TAG=${1:-r6cs}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $ROOT/tests/test_conv_gpu.py $ROOT/tests/test_unetr.py $ROOT/tests/test_upernet.py \
  $ROOT/tests/test_modules_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || { echo "STOP tests rc $rc"; exit 1; }
for r in 1 2; do
  for v in slots2 slots3; do
    echo "== $v round $r" >> $OUT/conv_ab.txt
    for set in c3 2d; do
      LCI_LIB_PATH=$ROOT/build_variants/liblci_$v.so timeout -k 10 300 python $ROOT/tools/conv_bench.py --set $set \
        --passes fwd,dgrad >> $OUT/conv_ab.txt 2>&1 || { echo "STOP conv $v $set"; exit 1; }
    done
  done
done
for v in slots2 slots3 slots2 slots3; do
  LCI_LIB_PATH=$ROOT/build_variants/liblci_$v.so timeout -k 10 400 python $ROOT/bench.py --workload swin_p2_128 --steps 10 \
    --warmup 3 --no-cpu-baseline > $OUT/c3_$v.json 2> $OUT/c3_$v.err || { echo "STOP bench $v"; tail -3 $OUT/c3_$v.err; exit 1; }
  python3 -c "import json; j=json.loads(open('$OUT/c3_$v.json').read().strip().splitlines()[-1]); k=j['kernels']; print('C3 $v', j['ms_per_step'], 'conv3', k.get('conv3'), 'wgrad', k.get('conv3_wgrad'))" | tee -a $OUT/c3_ab.txt
done
echo "r6_conv_slots_ab $TAG done"
