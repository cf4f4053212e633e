#!/bin/bash
# Round-6 records on one box: smoke, every workload's bench line (tools/bench_all_r5.sh), and the metric / C3
# rocprofv3 kernel traces with their FETCH_SIZE / WRITE_SIZE passes (tools/profile_r5.sh).
# Usage (GPU box): bash tools/r6_records.sh <tag>
TAG=${1:-r6}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $ROOT/gpurun_out/bench_$TAG
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $ROOT/gpurun_out/bench_$TAG/smoke.txt 2>&1 \
  || { echo "STOP smoke"; tail -5 $ROOT/gpurun_out/bench_$TAG/smoke.txt; exit 1; }
tail -1 $ROOT/gpurun_out/bench_$TAG/smoke.txt
bash $ROOT/tools/bench_all_r5.sh $TAG || exit 1
bash $ROOT/tools/profile_r5.sh $TAG metric c3 || exit 1
echo "records $TAG done"
