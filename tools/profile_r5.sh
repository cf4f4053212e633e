#!/bin/bash
# Round 5 profiles, each pass its own rocprofv3 run (counters in separate passes, no trace domains beside --pmc):
#   1. metric (vit_p2_512, --no-secondary): kernel trace + FETCH_SIZE / WRITE_SIZE     -> traffic.json vit_p2_512
#   2. C3 (swin_p2_128) eager (LCI_GRAPH=0: rocprofv3 --pmc aborts on graph replays, tools/graph_pmc_repro.py):
#      FETCH_SIZE / WRITE_SIZE                                                          -> traffic.json swin_p2_128
#   3. C4 FFT conv calls (tools/fft_traffic.py): FETCH_SIZE / WRITE_SIZE per call      -> traffic.json vit_hyena_p2_1024
# Usage (GPU box): bash tools/profile_r5.sh <tag> [stages...]  (stages: metric c3 c4 c5 fft wl-<workload>; default
# metric c3 fft)
TAG=$1; shift
STAGES=${*:-metric c3 fft}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
( while sleep 20; do date +%s >> $OUT/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
RE='attn_|conv3|scan_|fft|window|win_|hyena|dwconv|inorm|patch_embed|linear_|ln_|layernorm|gelu|upsample|gemm_bt|row_dot'
pmc() {   # pmc <dir> <counter> <cmd...>
  local d=$1 c=$2; shift 2
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --kernel-include-regex "$RE" --output-format csv -d $d -o run -- "$@" \
    > $d.log 2>&1 || { echo "STOP $d ($c)"; tail -5 $d.log; exit 1; }
  echo "$d done"
}
for st in $STAGES; do
  case $st in
    metric)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/metric/trace -o run -- \
        python3 $ROOT/bench.py --no-cpu-baseline --no-secondary --steps 5 --warmup 2 > $OUT/metric_trace.log 2>&1 \
        || { echo "STOP metric trace"; tail -5 $OUT/metric_trace.log; exit 1; }
      echo "metric trace done"
      mkdir -p $OUT/metric
      pmc $OUT/metric/fetch FETCH_SIZE python3 $ROOT/bench.py --no-cpu-baseline --no-secondary --no-kernel-timer --steps 3 --warmup 1
      pmc $OUT/metric/write WRITE_SIZE python3 $ROOT/bench.py --no-cpu-baseline --no-secondary --no-kernel-timer --steps 3 --warmup 1
      ;;
    c3)
      mkdir -p $OUT/c3
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3/trace -o run -- \
        python3 $ROOT/bench.py --workload swin_p2_128 --steps 5 --warmup 2 > $OUT/c3_trace.log 2>&1 \
        || { echo "STOP c3 trace"; tail -5 $OUT/c3_trace.log; exit 1; }
      echo "c3 trace done"
      export LCI_GRAPH=0
      pmc $OUT/c3/fetch FETCH_SIZE python3 $ROOT/bench.py --workload swin_p2_128 --no-kernel-timer --steps 3 --warmup 1
      pmc $OUT/c3/write WRITE_SIZE python3 $ROOT/bench.py --workload swin_p2_128 --no-kernel-timer --steps 3 --warmup 1
      unset LCI_GRAPH
      ;;
    c4|c5)   # vit_hyena_p2_1024 / vit_mamba_p2_256: trace + FETCH / WRITE passes of the workload (eager steps)
      WL=$([ $st = c4 ] && echo vit_hyena_p2_1024 || echo vit_mamba_p2_256)
      mkdir -p $OUT/$st
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$st/trace -o run -- \
        python3 $ROOT/bench.py --workload $WL --steps 3 --warmup 1 > $OUT/${st}_trace.log 2>&1 \
        || { echo "STOP $st trace"; tail -5 $OUT/${st}_trace.log; exit 1; }
      echo "$st trace done"
      pmc $OUT/$st/fetch FETCH_SIZE python3 $ROOT/bench.py --workload $WL --no-kernel-timer --steps 2 --warmup 1
      pmc $OUT/$st/write WRITE_SIZE python3 $ROOT/bench.py --workload $WL --no-kernel-timer --steps 2 --warmup 1
      ;;
    wl-*)   # any other workload (round 6): trace as it runs, FETCH / WRITE passes eager (LCI_GRAPH=0, as C3)
      WL=${st#wl-}
      mkdir -p $OUT/$WL
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$WL/trace -o run -- \
        python3 $ROOT/bench.py --workload $WL --steps 3 --warmup 2 > $OUT/${WL}_trace.log 2>&1 \
        || { echo "STOP $WL trace"; tail -5 $OUT/${WL}_trace.log; exit 1; }
      echo "$WL trace done"
      export LCI_GRAPH=0
      pmc $OUT/$WL/fetch FETCH_SIZE python3 $ROOT/bench.py --workload $WL --no-kernel-timer --steps 2 --warmup 1
      pmc $OUT/$WL/write WRITE_SIZE python3 $ROOT/bench.py --workload $WL --no-kernel-timer --steps 2 --warmup 1
      unset LCI_GRAPH
      ;;
    fft)
      mkdir -p $OUT/fft
      timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fft/fetch -o run -- \
        python3 $ROOT/tools/fft_traffic.py > $OUT/fft/fetch.log 2>&1 || { echo "STOP fft fetch"; exit 1; }
      timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/fft/write -o run -- \
        python3 $ROOT/tools/fft_traffic.py > $OUT/fft/write.log 2>&1 || { echo "STOP fft write"; exit 1; }
      echo "fft done"
      ;;
  esac
done
