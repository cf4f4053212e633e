#!/bin/bash
# Round-6 final GPU session: the full GPU suite, then tools/r6_records.sh (smoke, every workload's bench line, the
# metric / C3 rocprofv3 traces and FETCH / WRITE passes).
# Usage (GPU box): bash tools/r6_final.sh <tag>
TAG=${1:-r6f2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $ROOT/tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $ROOT/gpurun_out/$TAG/gputest.log 2>&1
rc=$?; tail -3 $ROOT/gpurun_out/$TAG/gputest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "STOP tests rc $rc"; exit 1; }
bash $ROOT/tools/r6_records.sh $TAG || exit 1
echo "final $TAG done"
