#!/bin/bash
# conv3 forward A/B: parity tests under the candidate kernel, then per-shape times of both kernels.
# Usage: bash tools/conv_ab.sh <tag> <ENV=VAL of the candidate> [sets...]
TAG=$1; CAND=$2; shift 2
SETS=${@:-c3 c5}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
env $CAND timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $OUT/test.log 2>&1
rc=$?; tail -3 $OUT/test.log; [ $rc -eq 0 ] || { echo "STOP tests rc $rc"; exit $rc; }
for s in $SETS; do
  timeout -k 10 400 python -u tools/conv_bench.py --passes ${PASSES:-fwd,dgrad} --set $s > $OUT/base_$s.jsonl 2>&1 || { echo "STOP base $s"; exit 1; }
  env $CAND timeout -k 10 400 python -u tools/conv_bench.py --passes ${PASSES:-fwd,dgrad} --set $s > $OUT/cand_$s.jsonl 2>&1 || { echo "STOP cand $s"; exit 1; }
done
python - "$OUT" $SETS <<'PY'
import json, sys
out = sys.argv[1]
for s in sys.argv[2:]:
    rows = {}
    for kind in ("base", "cand"):
        for l in open(f"{out}/{kind}_{s}.jsonl"):
            if l.startswith("{"):
                d = json.loads(l)
                rows.setdefault((tuple(d["S"]), d["cin"], d["cout"], d["pass"]), {})[kind] = d
    for k, v in rows.items():
        b, c = v.get("base", {}), v.get("cand", {})
        print(s, k, b.get("ms"), c.get("ms"), b.get("tflops"), c.get("tflops"))
PY
