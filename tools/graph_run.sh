#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/graph1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $ROOT/tests/test_graph_gpu.py -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/gputest.log | tail -3; [ $rc -le 1 ] || { echo "STOP tests rc $rc"; exit $rc; }
for w in swin_p2_128 swin_mamba_p2_128 swin_hyena_p2_128 vit_p4_512; do
  timeout -k 10 400 python -u $ROOT/bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  rc=$?; cut -c1-250 $OUT/bench_$w.json; [ $rc -eq 0 ] || { echo "STOP bench $w rc $rc"; tail -20 $OUT/bench_$w.err; exit $rc; }
done
echo graph1 done
