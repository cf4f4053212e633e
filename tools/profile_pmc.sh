#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs) of bench.py restricted to the liblci kernels, with a heartbeat file
# under gpurun_out/ while rocprofv3 collects. Usage (GPU box): bash tools/profile_pmc.sh <tag> [bench args...]
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
( while sleep 20; do date +%s >> $OUT/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
RE='attn_|conv3|scan_|fft|window|win_|hyena|dwconv|inorm|patch_embed|linear_|ln_|layernorm|gelu|upsample'
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 500 rocprofv3 --pmc $c --kernel-trace --kernel-include-regex "$RE" --output-format csv \
    -d $OUT/${c,,} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $OUT/${c,,}_bench.log 2>&1 \
    || { echo "STOP $c"; exit 1; }
  echo "$c done"
done
