#!/bin/bash
# Kernel-trace (--stats) pass + FETCH_SIZE / WRITE_SIZE passes (separate runs) of bench.py, with a heartbeat file
# under gpurun_out/ while rocprofv3 collects (a silent long pass reads as hung). Summarize afterwards with
# tools/summarize_prof.py. Usage (GPU box): [SKIP_TRACE=1] bash tools/profile_full.sh <tag> [bench args...]
# (counter passes need --no-secondary: the C3 line's HIP-graph replay aborts under rocprofv3 --pmc, 'AQL packet is
# malformed')
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
( while sleep 20; do date +%s >> $OUT/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
[ -n "$SKIP_TRACE" ] || timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $OUT/trace_bench.log 2>&1 || { echo "STOP trace"; exit 1; }
echo "trace done"
RE='attn_|conv3|scan_|fft|window|win_|hyena|dwconv|inorm|patch_embed|linear_|ln_|layernorm|gelu|upsample'
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 500 rocprofv3 --pmc $c --kernel-trace --kernel-include-regex "$RE" --output-format csv \
    -d $OUT/$([ $c = FETCH_SIZE ] && echo fetch || echo write) -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $OUT/${c,,}_bench.log 2>&1 \
    || { echo "STOP $c"; exit 1; }
  echo "$c done"
done
