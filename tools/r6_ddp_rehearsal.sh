#!/bin/bash
# The driver's N > 1 command path on one GPU: bench.py launched by torch.distributed.run with 2 ranks, gloo carrying
# DDP's all-reduce (LCI_DIST_BACKEND=gloo), both ranks on cuda:0 (bench.py maps LOCAL_RANK % device_count), the
# metric workload at full size. Checks that the N-rank line is produced (value = images of both ranks / max time).
# Usage (GPU box): bash tools/r6_ddp_rehearsal.sh <tag>
TAG=${1:-r6ddp}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
LCI_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 $ROOT/bench.py --gpus 2 --steps 3 --warmup 1 --no-secondary \
  > $OUT/bench_n2.json 2> $OUT/bench_n2.err || { echo "STOP n2"; tail -20 $OUT/bench_n2.err; exit 1; }
cut -c1-400 $OUT/bench_n2.json
echo "ddp rehearsal $TAG done"
