#!/bin/bash
# A/B of the Linear weight-gradient kernel: the in-tree library and build_variants/liblci_*.so (tools/attn_variants.sh
# build ...), each at a few workgroup targets (LCI_LW_WGS). Usage (GPU box): bash tools/lw_ab.sh [wgs ...]
WGS=${*:-512 2048}
for so in long_context_biomedical_imaging_amd/liblci.so build_variants/liblci_*.so; do
  [ -f $so ] || continue
  for w in $WGS; do
    echo "== $(basename $so) WGS $w"
    LCI_LIB_PATH=$PWD/$so LCI_LW_WGS=$w timeout -k 10 200 python -u tools/kernel_bench.py linear 2>&1 | grep linear_wgrad | cut -c1-100 || exit 1
  done
done
