#!/bin/bash
# One GPU-box session: GPU tests, the default bench line, a rocprofv3 kernel-trace summary of a short bench run,
# and PMC passes (one counter group per run, each under its own hard time limit). Any crash / time-out stops the
# script before the next GPU step; plain test failures (pytest rc 1) do not stop the bench.
# Usage (on the GPU box, from the repo root): bash tools/gpu_round.sh <tag> [tests|bench|trace|pmc ...]
TAG=$1; shift
STEPS=${*:-tests bench trace pmc}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc $2)"; exit $2; }
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest $ROOT/tests -m gpu -q --timeout 300 --timeout-method thread \
        -p no:cacheprovider > $OUT/gputest.log 2>&1
      rc=$?; tail -3 $OUT/gputest.log; [ $rc -le 1 ] || stop tests $rc ;;
    bench)
      timeout -k 10 600 python -u $ROOT/bench.py > $OUT/bench.json 2> $OUT/bench.err
      rc=$?; cat $OUT/bench.json | cut -c1-400; [ $rc -eq 0 ] || stop bench $rc ;;
    trace)
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
        -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > $OUT/trace_bench.json \
        2> $OUT/trace_bench.err)
      rc=$?; [ $rc -eq 0 ] || stop trace $rc ;;
    pmc)
      for grp in "FETCH_SIZE" "WRITE_SIZE" \
                 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
        name=$(echo $grp | cut -d' ' -f1)
        (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc_$name \
          -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-kernel-timer \
          > $OUT/pmc_$name.log 2>&1)
        rc=$?; tail -2 $OUT/pmc_$name.log; [ $rc -eq 0 ] || stop pmc_$name $rc
      done ;;
  esac
done
echo "gpu_round $TAG done"
