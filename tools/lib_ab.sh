#!/bin/bash
# Same-box A/B of liblci variants in build_variants/ (liblci_<name>.so), alternating, on one tools/ command.
# Usage (GPU box): bash tools/lib_ab.sh <tag> "<variant names>" <rounds> <command...>
TAG=$1; VARS=$2; R=$3; shift 3
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for v in $VARS; do
    echo "== $v round $r" >> $OUT/ab.txt
    LCI_LIB_PATH=$ROOT/build_variants/liblci_$v.so timeout -k 10 300 "$@" >> $OUT/ab.txt 2>&1 || { echo "STOP $v"; exit 1; }
  done
done
echo "lib_ab $TAG done"
