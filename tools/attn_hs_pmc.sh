#!/bin/bash
# SQ counters of the dK/dV kernel variants in build_variants/ (kernel_bench attention), one rocprofv3 pass per group.
# Usage (GPU box): bash tools/attn_hs_pmc.sh <tag> "<variants>"
TAG=${1:-hspmc}; VARS=${2:-"v2"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp LCI_NO_KTIMER=1
cd /tmp
for v in $VARS; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    LCI_LIB_PATH=$ROOT/build_variants/liblci_$v.so timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
      -d $OUT/${v}_pmc$i -o run -- python3 $ROOT/tools/kernel_bench.py attention > $OUT/${v}_pmc$i.log 2>&1 || exit 1
  done
  python3 $ROOT/tools/pmc_table.py $OUT/${v}_pmc1 $OUT/${v}_pmc2 @dkdv > $OUT/${v}_table.txt 2>&1
  echo "== $v"; cat $OUT/${v}_table.txt
done
