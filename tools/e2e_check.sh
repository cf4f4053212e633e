mkdir -p gpurun_out/r02e
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -x > gpurun_out/r02e/gputest.log 2>&1; tail -3 gpurun_out/r02e/gputest.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r02e/bench.json 2> gpurun_out/r02e/bench.err || exit 1
cut -c1-420 gpurun_out/r02e/bench.json
timeout -k 10 400 python -u bench.py --workload vit_mamba_p2_256 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r02e/c5.json 2> gpurun_out/r02e/c5.err || exit 1
cut -c1-300 gpurun_out/r02e/c5.json
