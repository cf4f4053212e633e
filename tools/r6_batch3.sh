#!/bin/bash
# Round 6: attention parity on the tree's library, a same-box attention A/B of build_variants, then the window
# backward's phase stamps (tools/r6_win_stamps.py, stamps variant).
# Usage (GPU box): bash tools/r6_batch3.sh <tag> "<variants>" <rounds>
TAG=$1; VARS=$2; R=${3:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PYT="python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PYT $ROOT/tests/test_attention_gpu.py $ROOT/tests/test_attention_long_gpu.py $ROOT/tests/test_gemm_small_gpu.py \
  $ROOT/tests/test_gemm_gpu.py $ROOT/tests/test_ddp_model_gpu.py $ROOT/tests/test_unetr.py $ROOT/tests/test_swin_alt_gpu.py > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "STOP tests rc $rc"; exit 1; }
[ -n "$VARS" ] && { bash $ROOT/tools/lib_ab.sh $TAG "$VARS" $R python $ROOT/tools/kernel_bench.py attention || exit 1; }
LCI_LIB_PATH=$ROOT/build_variants/liblci_stamps.so timeout -k 10 300 python -u $ROOT/tools/r6_win_stamps.py > $OUT/win_stamps.txt 2>&1 \
  || { echo "STOP stamps"; tail -5 $OUT/win_stamps.txt; exit 1; }
cat $OUT/win_stamps.txt
timeout -k 10 300 python -u $ROOT/tools/glue_time.py swin_p2_128 --rows 70 > $OUT/glue_c3.txt 2>&1 || { echo "STOP glue"; tail -5 $OUT/glue_c3.txt; exit 1; }
head -20 $OUT/glue_c3.txt
for sg in 0 1 0 1; do
  LCI_SMALL_GEMM=$sg timeout -k 10 300 python -u $ROOT/bench.py --workload swin_p2_128 --steps 10 --warmup 3 --no-cpu-baseline \
    > $OUT/c3_sg$sg.json 2>> $OUT/c3_sg.err || { echo "STOP c3 sg$sg"; tail -5 $OUT/c3_sg.err; exit 1; }
  echo "small_gemm=$sg $(cut -c1-200 $OUT/c3_sg$sg.json)"
done
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3trace -o run -- \
  python3 $ROOT/bench.py --workload swin_p2_128 --steps 4 --warmup 2 --no-cpu-baseline > $OUT/c3trace.log 2>&1) \
  || { echo "STOP c3 trace"; tail -5 $OUT/c3trace.log; exit 1; }
echo "batch3 $TAG done"
