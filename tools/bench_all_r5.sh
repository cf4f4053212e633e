#!/bin/bash
# Round-5 bench lines for every workload, one process each (GPU box): bash tools/bench_all_r5.sh <tag>
TAG=${1:-r5}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/bench_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_METRIC" ]; then
  timeout -k 10 900 python -u $ROOT/bench.py > $OUT/metric.json 2> $OUT/metric.err || { echo "STOP metric"; tail -5 $OUT/metric.err; exit 1; }
  echo "metric done"
fi
for wl in ${WORKLOADS:-vit_p4_512 vit_hyena_p2_1024 vit_hyena_p2_512 swin_mamba_p2_128 swin_hyena_p2_128 vit_mamba_p2_256}; do
  timeout -k 10 900 python -u $ROOT/bench.py --workload $wl --steps 5 --warmup 2 > $OUT/$wl.json 2> $OUT/$wl.err || { echo "STOP $wl"; tail -5 $OUT/$wl.err; exit 1; }
  echo "$wl done"
done
python3 - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print(os.path.basename(f), d["value"], d["ms_per_step"], r.get("kernel"), r.get("frac"), r.get("traffic"))
    for k, s in (d.get("secondary") or {}).items():
        rr = s.get("roofline", {})
        print("  secondary", k, s.get("value"), s.get("ms_per_step"), rr.get("kernel"), rr.get("frac"), rr.get("traffic"))
    if d.get("cpu_baseline"): print("  cpu", d["cpu_baseline"])
PY
