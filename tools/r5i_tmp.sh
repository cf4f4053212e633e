export TMPDIR=/tmp
OUT=gpurun_out/r5i
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_unetr.py tests/test_upernet.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/test.log 2>&1 || { echo "STOP test"; tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
timeout -k 10 600 python -u bench.py --workload swin_p2_128 --steps 10 --warmup 3 > $OUT/c3.json 2> $OUT/c3.err || { echo "STOP c3"; tail -3 $OUT/c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c3.json').read().strip().splitlines()[-1]); print('C3', d['ms_per_step'], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 1})"
timeout -k 10 600 python -u bench.py --workload vit_mamba_p2_256 --steps 5 --warmup 2 > $OUT/c5.json 2> $OUT/c5.err || { echo "STOP c5"; tail -3 $OUT/c5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c5.json').read().strip().splitlines()[-1]); print('C5', d['ms_per_step'], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 10})"
