#!/bin/bash
# One GPU call: scan A/B (tools/scan_ab_r5.sh) then the graph-replay PMC repro (torch-only graph first; the liblci
# graph only if that one completes). An abort ends the call (no further GPU step).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash $ROOT/tools/scan_ab_r5.sh scanab1 || exit 1
OUT=$ROOT/gpurun_out/graphpmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for m in torch lci; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/$m -o run -- python3 $ROOT/tools/graph_pmc_repro.py $m > $OUT/$m.log 2>&1
  rc=$?
  echo "graph pmc $m rc=$rc $(grep -h -E 'graph replay ok|malformed|rror' $OUT/$m.log | head -3)"
  [ $rc -eq 0 ] || exit 0
done
