#!/bin/bash
# Round-4 GPU test batch after the attention parity + A/B script: the given test files in one pytest process.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r4t}
shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest "$@" -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -s \
  > $OUT/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|^unetr|Error" $OUT/tests.log | tail -40
exit $rc
