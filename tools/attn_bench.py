"""Micro-benchmark of liblci flash attention fwd / bwd (HIP events, random N(0,1) bf16 data)."""
import argparse
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from long_context_biomedical_imaging_amd import kernels  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, nargs="+", default=[16384, 65536])
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--H", type=int, default=6)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    for L in a.L:
        qkv = torch.randn(a.B, L, 3 * a.H * 64, device="cuda").to(torch.bfloat16)
        dout = torch.randn(a.B, L, a.H * 64, device="cuda").to(torch.bfloat16)
        out, lse = kernels.attn_fwd(qkv, a.H, 0.125)
        tf = timeit(lambda: kernels.attn_fwd(qkv, a.H, 0.125), a.iters)
        tb = timeit(lambda: kernels.attn_bwd(qkv, out, dout, lse, a.H, 0.125), a.iters)
        f = 4.0 * a.B * a.H * L * L * 64
        print(json.dumps({"L": L, "B": a.B, "H": a.H, "fwd_ms": round(tf, 3), "bwd_ms": round(tb, 3),
                          "fwd_tflops": round(f / tf / 1e9, 1), "bwd_tflops_alg": round(2 * f / tb / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
