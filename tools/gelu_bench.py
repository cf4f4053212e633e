"""Time torch's bf16 GELU (fwd / bwd) against lci_gelu at the metric and C5 MLP shapes; prints ms and TB/s.
(profiles/r02_gelu_bench.txt also holds the measured, dropped variants: a fast-erf formula and a capped grid.)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from long_context_biomedical_imaging_amd import kernels  # noqa: E402


def t_ms(fn, it=20):
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
    tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("LCI_GELU"))
    for M in (131072, 1 << 21):
        x = torch.randn(M, 1536, device="cuda", dtype=torch.bfloat16)
        g = torch.randn_like(x)
        nb = x.numel() * 2
        f = {"torch_fwd": lambda: torch.nn.functional.gelu(x),
             "torch_bwd": lambda: torch.ops.aten.gelu_backward(g, x),
             "lci_fwd": lambda: kernels._GELU.forward(type("C", (), {"save_for_backward": lambda *a: None})(), x)}
        for name, fn in f.items():
            ms = t_ms(fn)
            nbytes = nb * (3 if "bwd" in name else 2)
            print(f"{tag:30s} M={M:8d} {name:10s} {ms:7.3f} ms {nbytes / ms / 1e9:5.2f} TB/s", flush=True)
        dx = torch.empty_like(x)
        from long_context_biomedical_imaging_amd import _lib
        ms = t_ms(lambda: _lib.call("lci_gelu_bwd", x.data_ptr(), g.data_ptr(), dx.data_ptr(), x.numel(),
                                    _lib.stream_of(x)))
        print(f"{tag:30s} M={M:8d} {'lci_bwd':10s} {ms:7.3f} ms {nb * 3 / ms / 1e9:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
