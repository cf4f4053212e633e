#!/bin/bash
# Round 6 batch (GPU box): the lse diagnostic, changed parity tests on the tree's library, an attention A/B of
# build_variants and the window-scan / scan-probe benches. Usage: bash tools/r6_batch.sh <tag>
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PYT="python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider"
for v in old rsum; do
  echo "== $v" >> $OUT/lse_diag.txt
  LCI_LIB_PATH=$ROOT/build_variants/liblci_$v.so timeout -k 10 300 python $ROOT/tools/r6_lse_diag.py >> $OUT/lse_diag.txt 2>&1 \
    || { echo "STOP diag"; exit 1; }
done
echo "diag done"
timeout -k 10 900 $PYT -x $ROOT/tests/test_mamba_gpu.py $ROOT/tests/test_optim_gpu.py $ROOT/tests/test_modules_gpu.py \
  $ROOT/tests/test_ddp_model_gpu.py $ROOT/tests/test_scan_long_gpu.py $ROOT/tests/test_swin_alt_gpu.py > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "STOP tests rc $rc"; exit 1; }
timeout -k 10 600 $PYT $ROOT/tests/test_attention_gpu.py $ROOT/tests/test_attention_long_gpu.py > $OUT/attn_test.log 2>&1
rc=$?; tail -3 $OUT/attn_test.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "STOP attn tests rc $rc"; exit 1; }
bash $ROOT/tools/lib_ab.sh $TAG "old rsum dqe" 2 python $ROOT/tools/kernel_bench.py attention || exit 1
for r in 1 2; do
  echo "== three-pass (LCI_SCAN_ONE=0 LCI_SCAN_PLAIN_DBC=0) round $r" >> $OUT/scan.txt
  LCI_SCAN_ONE=0 LCI_SCAN_PLAIN_DBC=0 timeout -k 10 300 python $ROOT/tools/kernel_bench.py scanwin >> $OUT/scan.txt 2>&1 \
    || { echo "STOP scanwin"; exit 1; }
  echo "== one-chunk round $r" >> $OUT/scan.txt
  timeout -k 10 300 python $ROOT/tools/kernel_bench.py scanwin >> $OUT/scan.txt 2>&1 || { echo "STOP scanwin"; exit 1; }
done
for v in tree probe; do
  echo "== long scan $v" >> $OUT/scan.txt
  lib=$ROOT/long_context_biomedical_imaging_amd/liblci.so; [ $v = probe ] && lib=$ROOT/build_variants/liblci_probe.so
  LCI_LIB_PATH=$lib timeout -k 10 300 python $ROOT/tools/kernel_bench.py scan >> $OUT/scan.txt 2>&1 \
    || { echo "STOP scan $v"; exit 1; }
done
echo "batch $TAG done"
