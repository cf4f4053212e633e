#!/bin/bash
# rocprofv3 kernel trace of the per-stage window-attention bench (tools/kernel_bench.py wstages).
# Usage (GPU box): bash tools/wprof.sh <tag> [env assignments...]
TAG=${1:-wprof}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for e in "$@"; do export "$e"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ROOT/tools/kernel_bench.py wstages > $OUT/trace.log 2>&1 || exit 1
echo "wprof $TAG done"
