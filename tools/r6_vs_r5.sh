#!/bin/bash
# Same-box A/B of the round-5 HEAD (665c198, staged by hand in build_variants/r05tree: its bench.py, package, built
# liblci.so and include/) against this tree: the metric step and the C3 step, alternating.
# Usage (GPU box): bash tools/r6_vs_r5.sh <tag>
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for v in r05 r06; do
    B=$ROOT/bench.py; [ $v = r05 ] && B=$ROOT/build_variants/r05tree/bench.py
    timeout -k 10 400 python -u $B --no-cpu-baseline --no-secondary --steps 6 --warmup 2 > $OUT/m_${v}_$r.json 2>> $OUT/err.txt \
      || { echo "STOP metric $v"; tail -5 $OUT/err.txt; exit 1; }
    echo "metric $v $(python3 -c "import json;d=json.loads(open('$OUT/m_${v}_$r.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
    timeout -k 10 300 python -u $B --workload swin_p2_128 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c3_${v}_$r.json 2>> $OUT/err.txt \
      || { echo "STOP c3 $v"; tail -5 $OUT/err.txt; exit 1; }
    echo "c3 $v $(python3 -c "import json;d=json.loads(open('$OUT/c3_${v}_$r.json').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
  done
done
echo "vs r5 $TAG done"
