"""Time the Hyena glue kernels (short conv + gates around the long conv) in isolation and report HBM rates.

Usage (GPU box): python tools/hyena_glue_bench.py [B L D heads K]   (default: the Hyena-512 layer, 2 65536 384 6 5)
Algorithmic bytes: pre_fwd  z (B,L,3D) bf16 in, vg (B,D,L) f32 + x2 (B,L,D) bf16 out
                   pre_bwd  z, dvg (B,D,L) f32, gx2 (B,L,D) f32 in, dz (B,L,3D) bf16 out
                   post_fwd y (B,D,L) f32, x2 in, out (B,L,D) bf16 out
                   post_bwd y, x2, dout (B,L,D) bf16 in, dy (B,D,L) f32 + dx2 (B,L,D) f32 out
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from long_context_biomedical_imaging_amd import _lib  # noqa: E402


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
    B, L, D, H, K = [int(a) for a in sys.argv[1:6]] if len(sys.argv) > 5 else (2, 65536, 384, 6, 5)
    hd = D // H
    dev = torch.device("cuda", 0)
    bf, f32 = torch.bfloat16, torch.float32
    z = torch.randn(B, L, 3 * D, device=dev, dtype=bf)
    w = torch.randn(3 * D, K, device=dev, dtype=f32)
    b = torch.randn(3 * D, device=dev, dtype=f32)
    vg = torch.empty(B, D, L, device=dev, dtype=f32)
    x2 = torch.empty(B, L, D, device=dev, dtype=bf)
    dvg = torch.randn(B, D, L, device=dev, dtype=f32)
    gx2 = torch.randn(B, L, D, device=dev, dtype=bf)   # ABI 26: the activation dtype
    dz = torch.empty_like(z)
    dw = torch.zeros(3 * D, K, device=dev, dtype=f32)
    db = torch.zeros(3 * D, device=dev, dtype=f32)
    y = torch.randn(B, D, L, device=dev, dtype=f32)
    out = torch.empty(B, L, D, device=dev, dtype=bf)
    dout = torch.randn(B, L, D, device=dev, dtype=bf)
    dy = torch.empty(B, D, L, device=dev, dtype=f32)
    dx2 = torch.empty(B, L, D, device=dev, dtype=bf)
    st = _lib.stream_of(z)
    n = B * L * D
    cases = {
        "pre_fwd": (lambda: _lib.call("lci_hyena_pre_fwd", 1, z.data_ptr(), w.data_ptr(), b.data_ptr(), vg.data_ptr(),
                                      x2.data_ptr(), B, L, H, hd, K, st), n * (3 * 2 + 4 + 2)),
        "pre_bwd": (lambda: _lib.call("lci_hyena_pre_bwd", 1, z.data_ptr(), w.data_ptr(), b.data_ptr(),
                                      dvg.data_ptr(), gx2.data_ptr(), dz.data_ptr(), dw.data_ptr(), db.data_ptr(),
                                      B, L, H, hd, K, st), n * (3 * 2 + 4 + 2 + 3 * 2)),
        "post_fwd": (lambda: _lib.call("lci_hyena_post_fwd", 1, y.data_ptr(), x2.data_ptr(), out.data_ptr(), B, L, D,
                                       st), n * (4 + 2 + 2)),
        "post_bwd": (lambda: _lib.call("lci_hyena_post_bwd", 1, y.data_ptr(), x2.data_ptr(), dout.data_ptr(),
                                       dy.data_ptr(), dx2.data_ptr(), B, L, D, st), n * (4 + 2 + 2 + 4 + 2)),
    }
    only = os.environ.get("GLUE_ONLY")
    for name, (fn, nbytes) in cases.items():
        if only and name not in only.split(","):
            continue
        ms = t_ms(fn)
        print(f"{name:9s} {ms * 1e3:8.1f} us  {nbytes / 1e6:7.1f} MB  {nbytes / ms / 1e9:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
