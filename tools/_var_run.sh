mkdir -p gpurun_out/r02d
for v in base prio rowc prio_rowc base; do
  so=build_variants/liblci_$v.so
  echo "== $v" >> gpurun_out/r02d/var.log
  LCI_LIB_PATH=$so timeout -k 10 200 python -m pytest tests/test_attention_gpu.py -q -x -p no:cacheprovider 2>&1 | tail -1 >> gpurun_out/r02d/var.log || exit 1
  LCI_LIB_PATH=$so timeout -k 10 200 python tools/kernel_bench.py attention >> gpurun_out/r02d/var.log 2>&1 || exit 1
done
cat gpurun_out/r02d/var.log
