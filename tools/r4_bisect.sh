for v in ${VARS:-a0s0}; do
  echo "== $v"; LCI_LIB_PATH=build_variants/liblci_$v.so timeout -k 10 120 python -m pytest tests/test_attention_gpu.py -m gpu -q -k "backward" -p no:cacheprovider 2>&1 | grep -E "passed|failed|AssertionError: d"
done
