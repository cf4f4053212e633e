#!/bin/bash
# Round 5: GPU suite + smoke + default bench line + kernel bench, each step under its own limit, stop on failure.
# Usage (GPU box): bash tools/gpu_r5.sh <tag> [kernel_bench groups...]   (SKIP_TESTS=1 / SKIP_BENCH=1 to skip)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5}; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $ROOT/tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
  rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || { echo "STOP tests rc $rc"; exit 1; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "STOP smoke"; tail -5 $OUT/smoke.log; exit 1; }
  echo smoke ok
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > $OUT/bench.json 2> $OUT/bench.err || { echo "STOP bench"; tail -5 $OUT/bench.err; exit 1; }
  python - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"], "roofline", d["roofline"]["kernel"], d["roofline"]["frac"], d["roofline"]["avg_launch_ms"])
for k in ("attn_fwd", "attn_bwd_dkdv", "attn_bwd_dq"):
    print(k, d["kernels"].get(k))
print("secondary", d.get("secondary", {}).get("swin_p2_128", {}).get("ms_per_step"))
PY
fi
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u tools/kernel_bench.py "$@" > $OUT/kbench.jsonl 2> $OUT/kbench.err || { echo "STOP kbench"; tail -5 $OUT/kbench.err; exit 1; }
  cat $OUT/kbench.jsonl
fi
