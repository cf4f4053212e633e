export TMPDIR=/tmp
OUT=gpurun_out/r5b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_c1_train_step_gpu.py tests/test_modules_gpu.py tests/test_gemm_gpu.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?
grep -E "C1|SGD|Adam|FAIL|Error|assert|passed|failed" $OUT/tests.log | tail -20
[ $rc -eq 0 ] || { echo "STOP tests rc=$rc"; exit 1; }
timeout -k 10 300 python -u tools/kernel_bench.py gemm > $OUT/gemm.jsonl 2> $OUT/gemm.err || { echo "STOP gemm bench"; tail -5 $OUT/gemm.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/gemm.jsonl'):
    d=json.loads(l); print(d['kernel'], d['config'].split(' bf16')[0], d['ms'], d['achieved'])
"
bash tools/gpu_r5_scan_graph.sh
