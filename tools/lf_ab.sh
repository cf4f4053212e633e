#!/bin/bash
# A/B of the fused-epilogue Linear GEMM (kernel_bench mlp): in-tree library and build_variants/liblci_*.so, each with
# LCI_LF_WIDE=0/1. Usage (GPU box): bash tools/lf_ab.sh
for so in long_context_biomedical_imaging_amd/liblci.so build_variants/liblci_*.so; do
  [ -f $so ] || continue
  for wide in 0 1; do
    echo "== $(basename $so) WIDE $wide"
    LCI_LIB_PATH=$PWD/$so LCI_LF_WIDE=$wide timeout -k 10 200 python -u tools/kernel_bench.py mlp 2>&1 | grep '"hip' | cut -c1-90 || exit 1
  done
done
