#!/bin/bash
# Round 6: small-GEMM parity + per-shape timing against hipBLASLt, the batch-coupling probe of the DDP test models,
# and the C3 step with / without the small GEMM.
# Usage (GPU box): bash tools/r6_batch4.sh <tag>
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PYT="python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PYT $ROOT/tests/test_gemm_small_gpu.py $ROOT/tests/test_window_gpu.py $ROOT/tests/test_window_index_gpu.py \
  $ROOT/tests/test_swin_alt_gpu.py $ROOT/tests/test_ddp_model_gpu.py $ROOT/tests/test_conv_gpu.py $ROOT/tests/test_unetr.py $ROOT/tests/test_sum_splits_gpu.py > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "STOP tests rc $rc"; exit 1; }
timeout -k 10 300 python -u $ROOT/tools/gemm_small_bench.py > $OUT/gemm_small.txt 2>&1 || { echo "STOP gemm bench"; tail -5 $OUT/gemm_small.txt; exit 1; }
cat $OUT/gemm_small.txt | grep -v amdgpu.ids
timeout -k 10 600 python -u $ROOT/tools/r6_batch_coupling.py > $OUT/coupling.txt 2>&1 || { echo "STOP coupling"; tail -5 $OUT/coupling.txt; exit 1; }
cat $OUT/coupling.txt | grep -v amdgpu.ids
for mb in 0 1 0 1; do
  LCI_WGRAD_MB3=$mb timeout -k 10 300 python -u $ROOT/tools/conv_bench.py --set c3 --passes wgrad > $OUT/wgrad_mb$mb.txt 2>&1 || { echo "STOP wgrad mb$mb"; exit 1; }
  echo "wgrad mb3=$mb"; grep -v amdgpu.ids $OUT/wgrad_mb$mb.txt | cut -c1-160
done
for sg in 0 1; do
  LCI_SMALL_GEMM=$sg timeout -k 10 300 python -u $ROOT/bench.py --workload swin_p2_128 --steps 10 --warmup 3 --no-cpu-baseline \
    > $OUT/c3_sg$sg.json 2>> $OUT/c3_sg.err || { echo "STOP c3 sg$sg"; tail -5 $OUT/c3_sg.err; exit 1; }
  echo "small_gemm=$sg $(cut -c1-200 $OUT/c3_sg$sg.json)"
done
for wo in 0 1 0 1; do
  LCI_WIN_ORDER=$wo timeout -k 10 300 python -u $ROOT/tools/kernel_bench.py wstages > $OUT/win_o$wo.txt 2>&1 || { echo "STOP win o$wo"; exit 1; }
  echo "win order $wo"; grep -v amdgpu.ids $OUT/win_o$wo.txt | cut -c1-150
done
echo "batch4 $TAG done"
