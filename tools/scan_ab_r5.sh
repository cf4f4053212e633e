#!/bin/bash
# Round 5 scan backward A/B (LCI_SCAN_BWD_V: 1 = round-4 kernel, 2 = packed-pair kernel, 3 = packed, 2 waves/SIMD)
# + parity at L = 2^21 + a kernel trace of the scan bench. Usage (GPU box): bash tools/scan_ab_r5.sh <tag>
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-scanab}
mkdir -p $OUT
export TMPDIR=/tmp
for v in 1 2 3 1 2 3; do
  LCI_SCAN_BWD_V=$v timeout -k 10 300 python -u tools/kernel_bench.py scan > $OUT/kb_v$v.jsonl 2>> $OUT/err.log || { echo "STOP kb v$v"; exit 1; }
  echo "v$v $(grep -h selective_scan_bwd $OUT/kb_v$v.jsonl | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms"], d["frac"])')"
done
for v in 2 3; do
  LCI_SCAN_BWD_V=$v timeout -k 10 600 python -u -m pytest tests/test_scan_long_gpu.py tests/test_mamba_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/test_v$v.log 2>&1 || { echo "STOP test v$v"; tail -20 $OUT/test_v$v.log; exit 1; }
  echo "tests v$v: $(tail -1 $OUT/test_v$v.log)"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ROOT/tools/kernel_bench.py scan > $OUT/trace.log 2>&1 || { echo "STOP trace"; exit 1; }
echo trace done
