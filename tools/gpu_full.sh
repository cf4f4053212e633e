#!/bin/bash
# Full GPU session: every -m gpu test, the default bench line (metric + C3 secondary + CPU baseline) and, optionally,
# extra workloads / tools. A crash or time-out stops the script; plain test failures (rc 1) do not stop the bench.
# Usage: bash tools/gpu_full.sh <tag> [workload ...]
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $ROOT/tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/gputest.log 2>&1
rc=$?; tail -5 $OUT/gputest.log; [ $rc -le 1 ] || { echo "STOP tests rc $rc"; exit $rc; }
timeout -k 10 600 python -u $ROOT/bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cut -c1-300 $OUT/bench.json; [ $rc -eq 0 ] || { echo "STOP bench rc $rc"; tail -20 $OUT/bench.err; exit $rc; }
for w in "$@"; do
  timeout -k 10 600 python -u $ROOT/bench.py --workload $w --no-cpu-baseline --steps 3 --warmup 2 \
    > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  rc=$?; cut -c1-200 $OUT/bench_$w.json; [ $rc -eq 0 ] || { echo "STOP bench $w rc $rc"; tail -20 $OUT/bench_$w.err; exit $rc; }
done
echo "gpu_full $TAG done"
