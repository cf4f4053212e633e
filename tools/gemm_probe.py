"""Time torch's (hipBLASLt) bf16 GEMMs for the Linear shapes of the workloads: forward Y = X W^T, data gradient
dX = dY W and weight gradient dW = dY^T X, at M tokens. Prints ms and TFLOP/s per (shape, form).
Usage (GPU box): python tools/gemm_probe.py [M ...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

SHAPES = {"qkv": (1152, 384), "proj": (384, 384), "fc1": (1536, 384), "fc2": (384, 1536),
          "m_in": (768, 384), "m_out": (384, 768), "m_x": (40, 192), "m_dt": (192, 24)}


def t_ms(fn, it=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def main():
    Ms = [int(a) for a in sys.argv[1:]] or [131072, 1 << 21]
    from long_context_biomedical_imaging_amd.trainer import use_tuned_gemms
    print("tuned table:", use_tuned_gemms())
    for M in Ms:
        for name, (N, K) in SHAPES.items():
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
            dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
            f = 2.0 * M * N * K
            res = []
            for form, fn in (("fwd", lambda: torch.nn.functional.linear(x, w)),
                             ("dgrad", lambda: dy @ w),
                             ("wgrad", lambda: dy.t() @ x)):
                ms = t_ms(fn)
                res.append(f"{form} {ms:7.3f} ms {f / ms / 1e9:6.0f} TF")
            print(f"M={M:8d} {name:6s} N={N:5d} K={K:5d} | " + " | ".join(res), flush=True)
            del x, w, dy
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
