"""Diagnostic: the forward's lse2 on the long-test input (late 4x-norm keys) against the exact fp64 lse, worst rows
with their (batch, head, row) and the row's query position within its 32-query block. Library via LCI_LIB_PATH."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from long_context_biomedical_imaging_amd import kernels  # noqa: E402
from oracle import attention as oatt  # noqa: E402

SCALE, LOG2E = 64 ** -0.5, 1.4426950408889634
B, L, H = 2, 65536, 6
C = H * 64
g = torch.Generator().manual_seed(65536)
qkv = torch.randn(B, L, 3 * C, generator=g)
for b, pos in ((0, 60001), (0, 65535), (1, 40000), (1, 65500)):
    qkv[b, pos, C:2 * C] *= 4.0
qkv = qkv.to(torch.bfloat16)
out, lse2 = kernels.attn_fwd(qkv.cuda(), H, SCALE)
lse2 = lse2.cpu().double()
q, k, v = oatt.split_qkv(qkv.float(), H)
rows = torch.tensor(sorted(set([0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 100, 101, 4095, 4096] +
                               torch.randint(0, L, (40,), generator=torch.Generator().manual_seed(1)).tolist())))
s = torch.einsum("bhid,bhjd->bhij", q[:, :, rows].double(), k.double()) * SCALE
lse = torch.logsumexp(s, -1)
got = lse2[:, :, rows] / LOG2E
dev = (got - lse)
print("max |dev|", dev.abs().max().item(), "mean |dev|", dev.abs().mean().item())
flat = dev.abs().flatten()
idx = flat.argsort(descending=True)[:12]
for i in idx.tolist():
    b, h, r = i // (H * len(rows)), (i // len(rows)) % H, i % len(rows)
    row = rows[r].item()
    print(f"b{b} h{h} row {row} (q%32={row % 32}) got {got[b, h, r].item():.5f} exact {lse[b, h, r].item():.5f} "
          f"dev {dev[b, h, r].item():+.2e}")
