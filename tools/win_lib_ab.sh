#!/bin/bash
# Window tests, then rocprofv3 kernel traces of the per-stage window bench for liblci variants (build_variants/).
# Usage (GPU box): bash tools/win_lib_ab.sh <tag> "<variants>"
TAG=$1; VARS=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $ROOT/tests/test_window_gpu.py $ROOT/tests/test_window_index_gpu.py $ROOT/tests/test_swin_alt_gpu.py -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
rc=$?; tail -1 $OUT/gputest.log; [ $rc -eq 0 ] || { echo "STOP tests rc $rc"; exit 1; }
cd /tmp
for r in 1 2; do for v in $VARS; do
  LCI_LIB_PATH=$ROOT/build_variants/liblci_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$v$r -o run -- python3 $ROOT/tools/kernel_bench.py wstages > $OUT/$v$r.log 2>&1 || exit 1
done; done
echo "win_lib_ab $TAG done"
