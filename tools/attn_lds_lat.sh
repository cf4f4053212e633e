#!/bin/bash
# Average LDS / VMEM instruction latency of the attention backward kernels (kernel_bench attention):
# SQ_ACCUM_PREV_HIRES accumulates the level counter just before it every cycle; latency = accumulated level / insts.
# Usage (GPU box): bash tools/attn_lds_lat.sh <tag> "<variants>"
TAG=${1:-ldslat}; VARS=${2:-"cur"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp LCI_NO_KTIMER=1
cd /tmp
for v in $VARS; do
  i=0
  for grp in "SQ_INST_LEVEL_LDS SQ_ACCUM_PREV_HIRES SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
             "SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    LCI_LIB_PATH=$ROOT/build_variants/liblci_$v.so timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
      -d $OUT/${v}_lat$i -o run -- python3 $ROOT/tools/kernel_bench.py attention > $OUT/${v}_lat$i.log 2>&1 || exit 1
  done
  echo "== $v"
  python3 $ROOT/tools/pmc_table.py $OUT/${v}_lat1 @attn_bwd
  python3 $ROOT/tools/pmc_table.py $OUT/${v}_lat2 @attn_bwd
done
