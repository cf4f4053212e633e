#!/bin/bash
# Build liblci variants of conv.hip (extra defines / flags) into build_variants/ here, then time them on the GPU
# box with tools/conv_bench.py:
#   bash tools/conv_variants.sh build "mv4:-DLCI_CONV_MV_WIDE=4" "agpr:-DLCI_CONV_MV_WIDE=4 NOVGPR" ...
#   bash tools/conv_variants.sh run [conv_bench args]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build_variants
CSRC=$ROOT/long_context_biomedical_imaging_amd/csrc
if [ "$1" = build ]; then
  shift
  mkdir -p $OUT
  python -m long_context_biomedical_imaging_amd.build_lib > /dev/null
  for spec in "$@"; do
    name=${spec%%:*}; defs=${spec#*:}
    vg="-Xarch_device -mllvm=-amdgpu-mfma-vgpr-form"
    case "$defs" in *NOVGPR*) vg=""; defs=${defs//NOVGPR/};; esac
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -munsafe-fp-atomics $vg $defs \
      -c $CSRC/conv.hip -o $OUT/cv_$name.conv.o
    objs=$(ls $CSRC/build/*.o | grep -v conv.hip.o)
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $OUT/cv_$name.conv.o -o $OUT/liblci_cv_$name.so
    echo "built $OUT/liblci_cv_$name.so ($defs $vg)"
  done
elif [ "$1" = run ]; then
  shift
  for so in $OUT/liblci_cv_*.so; do
    echo "== $so"
    LCI_LIB_PATH=$so timeout -k 10 200 python -u $ROOT/tools/conv_bench.py "$@"
  done
fi
