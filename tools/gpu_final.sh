set -o pipefail
OUT=gpurun_out/${FINAL_TAG:-r02w}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1; rc=$?; tail -3 $OUT/gputest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --workload vit_mamba_p2_256 --steps 3 --warmup 2 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; cut -c1-300 $OUT/bench_c5.json; exit $rc
