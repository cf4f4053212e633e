#!/bin/bash
# Window-attention GPU check: the window tests, then the per-stage bench with the single-phase backward (default)
# and the two-phase kernel (LCI_WIN_BWD1=0). Usage (GPU box): bash tools/win_ab.sh <tag>
TAG=${1:-win}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $ROOT/tests/test_window_gpu.py $ROOT/tests/test_window_index_gpu.py -m gpu -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/gputest.log | tail -3; [ $rc -le 1 ] || { echo "STOP tests rc $rc"; exit $rc; }
timeout -k 10 300 python -u $ROOT/tools/kernel_bench.py wstages > $OUT/wstages_bwd1.jsonl 2>&1 || exit 1
LCI_WIN_BWD1=0 timeout -k 10 300 python -u $ROOT/tools/kernel_bench.py wstages > $OUT/wstages_bwd2.jsonl 2>&1 || exit 1
LCI_WIN_FWD_NW=8 timeout -k 10 300 python -u $ROOT/tools/kernel_bench.py wstages > $OUT/wstages_fwd8.jsonl 2>&1 || exit 1
echo "win_ab $TAG done"
