#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/c5ck
mkdir -p $OUT
for k in 11 10; do
  timeout -k 10 400 python -u $ROOT/bench.py --workload vit_mamba_p2_256 --steps 3 --warmup 2 --no-cpu-baseline --ckpt-blocks $k > $OUT/bench_ck$k.json 2> $OUT/bench_ck$k.err
  rc=$?; cut -c1-200 $OUT/bench_ck$k.json; [ $rc -eq 0 ] || { echo "ck$k rc $rc"; tail -3 $OUT/bench_ck$k.err; }
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
echo c5ck done
