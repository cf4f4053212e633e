export TMPDIR=/tmp
OUT=gpurun_out/r5k
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_window_gpu.py tests/test_swin_alt_gpu.py tests/test_window_index_gpu.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/test.log 2>&1 || { echo "STOP test"; tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
timeout -k 10 300 python -u tools/kernel_bench.py window > $OUT/kb.jsonl 2> $OUT/kb.err || { echo "STOP kb"; tail $OUT/kb.err; exit 1; }
cat $OUT/kb.jsonl | cut -c1-200
timeout -k 10 600 python -u bench.py --workload swin_p2_128 --steps 10 --warmup 3 > $OUT/c3.json 2> $OUT/c3.err || { echo "STOP c3"; tail -3 $OUT/c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c3.json').read().strip().splitlines()[-1]); print('C3', d['ms_per_step'], d['roofline']['frac'], {k: v for k, v in d['kernels'].items() if 'window' in k})"
bash tools/pmc_r5.sh pmc_r5w2 window || exit 1
