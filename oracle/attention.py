"""Oracle: ViT full self-attention (SABlock), CPU restatement. Test infrastructure only.

Follows /root/reference/model/models/backbone_vit.py:
  :166-169  qkv Linear (bias=qkv_bias), out_proj Linear(bias), Rearrange "b h (qkv l d) -> qkv b l h d"
  :191-203  q,k,v; att = softmax(einsum(q,k)*scale); x = einsum(att, v); "b h l d -> b l (h d)"; out_proj
"""
from __future__ import annotations

import math

import torch


def split_qkv(qkv: torch.Tensor, num_heads: int):
    """(B, L, 3*D) -> q, k, v each (B, H, L, Dh). Channel order (qkv, head, d) (backbone_vit.py:168)."""
    b, l, three_d = qkv.shape
    dh = three_d // (3 * num_heads)
    t = qkv.reshape(b, l, 3, num_heads, dh).permute(2, 0, 3, 1, 4)
    return t[0], t[1], t[2]


def attention_core(q, k, v, scale: float, q_chunk: int | None = None):
    """o[b,h,x,:] = softmax_y(q[x].k[y]*scale) @ v (backbone_vit.py:193,200).

    q_chunk: compute query rows in chunks (per-row softmax, so exact) to bound memory at large L.
    Returns (o, lse) with lse = natural-log logsumexp of the scaled scores per query row.
    """
    L = q.shape[-2]
    q_chunk = q_chunk or L
    outs, lses = [], []
    for s in range(0, L, q_chunk):
        sc = torch.einsum("blxd,blyd->blxy", q[..., s:s + q_chunk, :], k) * scale
        lse = torch.logsumexp(sc, dim=-1)
        att = sc.softmax(dim=-1)
        outs.append(torch.einsum("bhxy,bhyd->bhxd", att, v))
        lses.append(lse)
    return torch.cat(outs, dim=-2), torch.cat(lses, dim=-1)


def sablock_attention(x, qkv_w, qkv_b, out_w, out_b, num_heads: int, q_chunk: int | None = None):
    """SABlock.forward attention branch (backbone_vit.py:191-203), dropout p=0."""
    qkv = torch.nn.functional.linear(x, qkv_w, qkv_b)
    q, k, v = split_qkv(qkv, num_heads)
    dh = q.shape[-1]
    o, _ = attention_core(q, k, v, dh ** -0.5, q_chunk)
    o = o.permute(0, 2, 1, 3).reshape(x.shape[0], x.shape[1], -1)
    return torch.nn.functional.linear(o, out_w, out_b)


def attention_flops_fwd_bwd(B: int, H: int, L: int, dh: int) -> float:
    """Algorithmic FLOPs of QK^T + AV, fwd (4*B*H*L^2*dh) + bwd (8*B*H*L^2*dh)."""
    return 12.0 * B * H * L * L * dh


def attention_flops_fwd(B: int, H: int, L: int, dh: int) -> float:
    return 4.0 * B * H * L * L * dh


__all__ = ["split_qkv", "attention_core", "sablock_attention", "attention_flops_fwd_bwd",
           "attention_flops_fwd", "math"]
