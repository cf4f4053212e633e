#!/bin/bash
# Build liblci variants of attention.hip / window.hip with extra defines into build_variants/ (run here, before gpurun),
# or time them on the GPU box:  bash tools/attn_variants.sh build "v1:-DLCI_IGLP=0" ... ; bash tools/attn_variants.sh run
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build_variants
if [ "$1" = build ]; then
  shift
  mkdir -p $OUT
  for spec in "$@"; do
    name=${spec%%:*}; defs=${spec#*:}
    objs=""
    for f in $ROOT/long_context_biomedical_imaging_amd/csrc/*.hip $ROOT/long_context_biomedical_imaging_amd/csrc/*.cpp; do
      b=$(basename $f)
      extra=""
      case $b in attention.hip) extra="-fno-honor-nans -fno-slp-vectorize $defs";; window.hip) extra="-fno-honor-nans $defs";; *.hip) extra="$defs";; esac
      if [ "${b##*.}" = hip ]; then
        /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -munsafe-fp-atomics \
          -Xarch_device -mllvm=-amdgpu-mfma-vgpr-form $extra -c $f -o $OUT/$name.$b.o &
      else
        /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I $ROOT/include -c $f -o $OUT/$name.$b.o &
      fi
      objs="$objs $OUT/$name.$b.o"
    done
    wait
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs -o $OUT/liblci_$name.so
    echo "built $OUT/liblci_$name.so ($defs)"
  done
elif [ "$1" = run ]; then
  which=${2:-attention}   # kernel_bench.py section: attention | window | ...
  for so in $OUT/liblci_*.so; do
    echo "== $(basename $so)"
    LCI_LIB_PATH=$so timeout -k 10 200 python $ROOT/tools/kernel_bench.py $which
  done
fi
