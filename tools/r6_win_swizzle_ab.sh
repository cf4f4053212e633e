#!/bin/bash
# Round 6: swizzled window-attention LDS tiles (r6v: t0 / t1 and the bwd1 scratch; r6w: the scratch only) -- window / Swin parity on the tree's library, then a same-box A/B of
# build_variants liblci_winnew (the tree) and liblci_winold (HEAD's window.hip): kernel_bench window, SQ pass of both,
# and the C3 bench line. Usage (GPU box): bash tools/r6_win_swizzle_ab.sh <tag>
TAG=${1:-r6ws}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $ROOT/tests/test_window_gpu.py $ROOT/tests/test_window_index_gpu.py \
  $ROOT/tests/test_swin_alt_gpu.py $ROOT/tests/test_unetr.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || { echo "STOP tests rc $rc"; exit 1; }
bash $ROOT/tools/lib_ab.sh $TAG "winold winnew" 3 python $ROOT/tools/kernel_bench.py window || exit 1
cd /tmp
for v in winold winnew; do
  LCI_NO_KTIMER=1 LCI_LIB_PATH=$ROOT/build_variants/liblci_$v.so timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace \
    --output-format csv -d $OUT/${v}_pmc2 -o run -- python3 $ROOT/tools/kernel_bench.py window > $OUT/${v}_pmc2.log 2>&1 || { echo "STOP pmc $v"; exit 1; }
  LCI_NO_KTIMER=1 LCI_LIB_PATH=$ROOT/build_variants/liblci_$v.so timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES \
    SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace \
    --output-format csv -d $OUT/${v}_pmc1 -o run -- python3 $ROOT/tools/kernel_bench.py window > $OUT/${v}_pmc1.log 2>&1 || { echo "STOP pmc1 $v"; exit 1; }
  python3 $ROOT/tools/pmc_table.py $OUT/${v}_pmc1 $OUT/${v}_pmc2 @win > $OUT/${v}_table.txt 2>&1
done
cd $ROOT
for v in winold winnew winold winnew; do
  LCI_LIB_PATH=$ROOT/build_variants/liblci_$v.so timeout -k 10 400 python $ROOT/bench.py --workload swin_p2_128 --steps 10 \
    --warmup 3 --no-cpu-baseline > $OUT/c3_$v.json 2> $OUT/c3_$v.err || { echo "STOP bench $v"; tail -3 $OUT/c3_$v.err; exit 1; }
  python3 -c "import json; j=json.loads(open('$OUT/c3_$v.json').read().strip().splitlines()[-1]); k=j['kernels']; print('C3 $v', j['ms_per_step'], {n: k[n]['ms_per_step'] for n in k if 'win' in n})" | tee -a $OUT/c3_ab.txt
done
echo "r6_win_swizzle_ab $TAG done"
