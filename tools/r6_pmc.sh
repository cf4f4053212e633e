#!/bin/bash
# Round-6 SQ counter passes of the production library (tools/pmc_r5.sh groups): attention and window attention
# (tools/kernel_bench.py), then the conv kernels at one C3 and one C5 shape (tools/conv_pmc.sh), with per-kernel tables.
# Usage (GPU box): bash tools/r6_pmc.sh <tag>
TAG=${1:-r6pmc}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
bash $ROOT/tools/pmc_r5.sh $TAG attention window > $OUT/sq.txt 2>&1 || { echo "STOP sq"; tail -5 $OUT/sq.txt; exit 1; }
for s in "c3 96-96" "c5 256-256"; do
  set -- $s
  bash $ROOT/tools/conv_pmc.sh $TAG/conv_$1 $2 $1 > $OUT/conv_$1.log 2>&1 || { echo "STOP conv $1"; tail -5 $OUT/conv_$1.log; exit 1; }
  python3 $ROOT/tools/pmc_table.py $OUT/conv_$1/pmc1 $OUT/conv_$1/pmc2 @conv3 > $OUT/conv_$1/table.txt 2>&1
done
echo "r6_pmc $TAG done"
