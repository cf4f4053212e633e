#!/bin/bash
# Round-5 SQ counter passes (MFMA / VALU busy, waits, LDS) of the production library's kernels under
# tools/kernel_bench.py <group>, one rocprofv3 run per counter group. Usage (GPU box): bash tools/pmc_r5.sh <tag> <group...>
TAG=${1:-pmc_r5}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp LCI_NO_KTIMER=1
cd /tmp
for g in "$@"; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
      -d $OUT/${g}_pmc$i -o run -- python3 $ROOT/tools/kernel_bench.py $g > $OUT/${g}_pmc$i.log 2>&1 || { echo "STOP $g $i"; tail -5 $OUT/${g}_pmc$i.log; exit 1; }
  done
  python3 $ROOT/tools/pmc_table.py $OUT/${g}_pmc1 $OUT/${g}_pmc2 @lci > $OUT/${g}_table.txt 2>&1
  echo "== $g"; cat $OUT/${g}_table.txt
done
