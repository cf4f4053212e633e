#!/bin/bash
# rocprofv3 passes over tools/kernel_bench.py sections: kernel trace, FETCH_SIZE, WRITE_SIZE and an SQ counter pass
# (one group per run, each under a hard limit). Usage (GPU box): bash tools/prof_kernels.sh <tag> <section...>
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
for sec in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$sec/trace -o run -- python3 $ROOT/tools/kernel_bench.py $sec > $OUT/$sec.trace.log 2>&1 || exit 1
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
    name=$(echo $grp | cut -d' ' -f1)
    LCI_NO_KTIMER=1 timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/$sec/pmc_$name -o run -- python3 $ROOT/tools/kernel_bench.py $sec > $OUT/$sec.pmc_$name.log 2>&1 || exit 1
  done
done
echo "prof_kernels $TAG done"
