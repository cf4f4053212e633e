"""lci_gemm_bt_small against hipBLASLt (torch.nn.functional.linear, bf16) on the C3 projection / 1x1-conv shapes.

HIP events around 20 back-to-back calls of each; one JSON line per shape: ms of both and the ratio. The product
routing in kernels.gemm_small_preferred comes from these lines (profiles/r06_gemm_small.txt).
Usage (GPU box): python tools/gemm_small_bench.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from long_context_biomedical_imaging_amd import kernels  # noqa: E402

# (M, N, K): Swin-tiny + SwinUNETR at 128^3 p2 (C3), forward and data-gradient GEMMs of the Linear layers lci_gemm_bt
# does not take, and the decoder's 1x1 convolutions
SHAPES = [
    (262144, 288, 96), (262144, 96, 96), (262144, 96, 384), (262144, 96, 288),
    (32768, 576, 192), (32768, 192, 192), (32768, 192, 768), (32768, 192, 576),
    (4096, 1152, 384), (4096, 384, 384), (4096, 1536, 384), (4096, 384, 1536), (4096, 384, 1152),
    (512, 2304, 768), (512, 768, 768), (512, 3072, 768), (512, 768, 3072), (512, 768, 2304),
    (2097152, 96, 192), (2097152, 192, 96), (2097152, 96, 96), (262144, 192, 192), (262144, 96, 192),
]


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    torch.manual_seed(0)
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        b = torch.randn(N, device="cuda").to(torch.bfloat16)
        ts = timeit(lambda: kernels.gemm_small(x, w, b))
        tb = timeit(lambda: torch.nn.functional.linear(x, w, b))
        fl = 2.0 * M * N * K
        byt = 2.0 * (M * K + M * N + N * K)
        print(json.dumps({"M": M, "N": N, "K": K, "small_ms": round(ts, 4), "hipblaslt_ms": round(tb, 4),
                          "ratio": round(tb / ts, 2), "small_tflops": round(fl / ts / 1e9, 1),
                          "small_gbs": round(byt / ts / 1e6, 1)}), flush=True)
        del x, w, b


if __name__ == "__main__":
    main()
