#!/usr/bin/env python3
"""Segment timing of the one-wave-per-SIMD dK/dV kernel from a diagnostic build (-DLCI_HS_STAMP=1, LCI_LIB_PATH):
s_memtime at the start of each of the 8 segments of tiles 64-95 (workgroups 0-7) and around the tile barrier.
Prints the median cycles per segment (ideal: 8 MFMAs x 32 = 256) and of the barrier."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from long_context_biomedical_imaging_amd import _lib, kernels  # noqa: E402

B, H, L = 2, 6, 65536
qkv = torch.randn(B, L, 3 * H * 64, device="cuda").to(torch.bfloat16)
dout = torch.randn(B, L, H * 64, device="cuda").to(torch.bfloat16)
out, lse = kernels.attn_fwd(qkv, H, 0.125)
dqkv = torch.zeros_like(qkv)
ws = torch.empty(int(_lib.load().lci_attn_bwd_ws_bytes(B, H, L)), device="cuda", dtype=torch.uint8)
args = (qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), dqkv.data_ptr(), ws.data_ptr(),
        B, L, H, 64, 0.125, _lib.stream_of(qkv))
_lib.call("lci_attn_bwd_stage", 0, *args)
for _ in range(3):
    _lib.call("lci_attn_bwd_stage", 1, *args)
torch.cuda.synchronize()
raw = dqkv.view(torch.uint8).flatten()[: 8 * 4 * 32 * 10 * 8].cpu().numpy().view(np.uint64).astype(np.int64)
st = raw.reshape(8, 4, 32, 10)
names = ["h0 segA", "h0 segB", "h0 segC", "h0 segD", "h1 segA", "stage", "h1 segB", "h1 segC", "h1 segD"]
# order in time: 0 1 2 3 4 [8 9] 5 6 7, next tile's 0
seq = [0, 1, 2, 3, 4, 8, 9, 5, 6, 7]
d = []
for i in range(len(seq) - 1):
    d.append(st[..., seq[i + 1]] - st[..., seq[i]])
nxt = st[:, :, 1:, 0] - st[:, :, :-1, 7]
labels = ["h0 A", "h0 B", "h0 C", "h0 D", "h1 A", "vmcnt->barrier", "h1 B(after bar)", "h1 C"]
for lab, x in zip(labels, d):
    print(f"{lab:18s} median {int(np.median(x)):6d}  p90 {int(np.percentile(x, 90)):6d}")
print(f"{'h1 D':18s} median {int(np.median(nxt)):6d}  p90 {int(np.percentile(nxt, 90)):6d}")
tile = st[:, :, 1:, 0] - st[:, :, :-1, 0]
print(f"tile total         median {int(np.median(tile)):6d}  (64 MFMAs x 32 = 2048 ideal)")
