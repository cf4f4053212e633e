#!/bin/bash
# rocprofv3 kernel trace of a few training steps of one bench workload (every kernel: liblci, hipBLASLt, torch).
# Usage (GPU box): bash tools/prof_step.sh <tag> <workload> [steps]
TAG=$1; W=$2; N=${3:-3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ROOT/bench.py --workload $W --steps $N --warmup 2 --no-cpu-baseline --no-secondary > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo "prof_step $TAG done"
