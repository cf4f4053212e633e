#!/bin/bash
# Round-3 GPU session helper: selected GPU test files and short bench runs of selected workloads, each step under
# its own time limit; a crash / time-out stops the script (plain test failures, rc 1, do not).
# Usage: bash tools/gpu_r3.sh <tag> "<test files or empty>" "<workloads or empty>" [bench extra args]
TAG=$1; TESTS=$2; WLS=$3; shift 3
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/gputest.log 2>&1
  rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/gputest.log | tail -40; [ $rc -le 1 ] || { echo "STOP tests rc $rc"; exit $rc; }
fi
for w in $WLS; do
  timeout -k 10 600 python -u $ROOT/bench.py --workload $w --no-cpu-baseline --no-secondary "$@" \
    > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  rc=$?; cut -c1-600 $OUT/bench_$w.json; [ $rc -eq 0 ] || { echo "STOP bench $w rc $rc"; tail -20 $OUT/bench_$w.err; exit $rc; }
done
echo "gpu_r3 $TAG done"
