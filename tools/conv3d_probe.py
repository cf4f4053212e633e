"""Time the 3-D conv / transposed-conv / instance-norm ops of the SwinUNETR head at 128^3 (patch 2) one by one.

Diagnostic for the decoder heads: prints each op's first-call time (MIOpen find /
kernel build included) and its steady-state fwd+bwd time, flushing after every op so a slow solver is named.
Usage (GPU box): python tools/conv3d_probe.py [--layout ncdhw|ndhwc] [--size 128]
"""
import argparse
import time

import torch
import torch.nn as nn

import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from long_context_biomedical_imaging_amd import decoders  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--layout", default="ncdhw", choices=["ncdhw", "ndhwc"])
ap.add_argument("--size", type=int, default=128)
ap.add_argument("--only", default="")
ap.add_argument("--hip", action="store_true", help="the repo's decoder convs (HIP conv3 / GEMM forms)")
args = ap.parse_args()
S = args.size
dev = torch.device("cuda")
# (name, module ctor, input shape): the SwinUNETR head's distinct conv shapes at S^3, patch 2 (Swin-tiny)
cases = [
    ("conv1to96_k3", lambda: nn.Conv3d(1, 96, 3, 1, 1, bias=False), (1, 1, S, S, S)),
    ("conv96to96_k3_S", lambda: nn.Conv3d(96, 96, 3, 1, 1, bias=False), (1, 96, S, S, S)),
    ("conv192to96_k3_S", lambda: nn.Conv3d(192, 96, 3, 1, 1, bias=False), (1, 192, S, S, S)),
    ("conv192to96_k1_S", lambda: nn.Conv3d(192, 96, 1, 1, 0, bias=False), (1, 192, S, S, S)),
    ("convT96_k2_S/2", lambda: nn.ConvTranspose3d(96, 96, 2, 2, bias=False), (1, 96, S // 2, S // 2, S // 2)),
    ("conv96to96_k3_S/2", lambda: nn.Conv3d(96, 96, 3, 1, 1, bias=False), (1, 96, S // 2, S // 2, S // 2)),
    ("conv192_k3_S/4", lambda: nn.Conv3d(192, 192, 3, 1, 1, bias=False), (1, 192, S // 4, S // 4, S // 4)),
    ("conv768to384_k3_S/16", lambda: nn.Conv3d(768, 384, 3, 1, 1, bias=False), (1, 768, S // 16, S // 16, S // 16)),
    ("conv1536_k3_S/32", lambda: nn.Conv3d(1536, 1536, 3, 1, 1, bias=False), (1, 1536, S // 32, S // 32, S // 32)),
    ("inorm96_S", lambda: nn.InstanceNorm3d(96), (1, 96, S, S, S)),
    ("out96to2_k1_S", lambda: nn.Conv3d(96, 2, 1, 1, 0, bias=True), (1, 96, S, S, S)),
]
mf = torch.channels_last_3d if args.layout == "ndhwc" else torch.contiguous_format
print(f"layout={args.layout} S={S}", flush=True)
for name, ctor, shape in cases:
    if args.only and args.only not in name:
        continue
    m = ctor()
    if args.hip and isinstance(m, (nn.Conv3d, nn.ConvTranspose3d)):
        k, st = m.kernel_size, m.stride
        hm = decoders._conv(3, m.in_channels, m.out_channels, k, st,
                            transposed=isinstance(m, nn.ConvTranspose3d), bias=m.bias is not None)
        hm.load_state_dict(m.state_dict())
        m = hm
    m = m.to(dev).to(memory_format=mf)
    x = torch.randn(shape, device=dev).to(memory_format=mf).requires_grad_(True)
    times = []
    for it in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        y.float().sum().backward()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t)
        print(f"  {name} call {it}: {times[-1] * 1e3:.1f} ms", flush=True)
    print(f"{name}: first {times[0]:.2f} s, steady {times[-1] * 1e3:.2f} ms", flush=True)
    del m, x, y
