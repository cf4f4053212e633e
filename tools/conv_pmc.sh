#!/bin/bash
# Conv kernels at one C5 shape: timing, kernel trace and two SQ counter passes.
# Usage (GPU box): bash tools/conv_pmc.sh <tag> <cin-cout> [set]
TAG=$1; ONLY=$2; SET=${3:-c5}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp LCI_NO_KTIMER=1
cd /tmp
timeout -k 10 300 python3 $ROOT/tools/conv_bench.py --set $SET --only $ONLY > $OUT/conv_bench.jsonl 2> $OUT/conv_bench.err || exit 1
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc$i -o run -- python3 $ROOT/tools/conv_bench.py --set $SET --only $ONLY --reps 2 > $OUT/pmc$i.log 2>&1 || exit 1
done
echo "conv_pmc $TAG done"
