"""torch.autograd wrappers over the liblci C-ABI. Each op runs the HIP kernels; none has a CPU path."""
from __future__ import annotations

import torch

from . import _lib


# ------------------------------------------------------------------------------------- attention
def attn_fwd(qkv: torch.Tensor, num_heads: int, scale: float):
    """qkv (B, L, 3*H*64) bf16 -> out (B, L, H*64) bf16, lse2 (B, H, L) f32."""
    _lib.require_gpu(qkv)
    B, L, C = qkv.shape
    dh = C // (3 * num_heads)
    if qkv.dtype != torch.bfloat16:
        raise _lib.LciError("attn_fwd expects bf16 qkv")
    out = torch.empty(B, L, num_heads * dh, device=qkv.device, dtype=torch.bfloat16)
    lse2 = torch.empty(B, num_heads, L, device=qkv.device, dtype=torch.float32)
    _lib.call("lci_attn_fwd", qkv.data_ptr(), out.data_ptr(), lse2.data_ptr(), B, L, num_heads, dh,
              float(scale), _lib.stream_of(qkv))
    return out, lse2


def attn_bwd(qkv, out, dout, lse2, num_heads: int, scale: float):
    _lib.require_gpu(qkv, out, dout, lse2)
    B, L, C = qkv.shape
    dh = C // (3 * num_heads)
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B, num_heads, L, device=qkv.device, dtype=torch.float32)
    _lib.call("lci_attn_bwd", qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse2.data_ptr(),
              dqkv.data_ptr(), delta.data_ptr(), B, L, num_heads, dh, float(scale), _lib.stream_of(qkv))
    return dqkv


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, num_heads, scale):
        out, lse2 = attn_fwd(qkv, num_heads, scale)
        ctx.save_for_backward(qkv, out, lse2)
        ctx.num_heads, ctx.scale = num_heads, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse2 = ctx.saved_tensors
        dout = dout.to(torch.bfloat16).contiguous()
        return attn_bwd(qkv, out, dout, lse2, ctx.num_heads, ctx.scale), None, None


def flash_attention(qkv: torch.Tensor, num_heads: int, scale: float) -> torch.Tensor:
    """softmax(q k^T * scale) v for the packed qkv projection (B, L, 3*H*dh) -> (B, L, H*dh).

    Computes in bf16 MFMA with f32 accumulation and f32 softmax. A non-bf16 qkv (no autocast) is cast to
    bf16 for the kernel and the result cast back.
    """
    dt = qkv.dtype
    q = qkv if dt == torch.bfloat16 else qkv.to(torch.bfloat16)
    o = _FlashAttention.apply(q.contiguous(), num_heads, scale)
    return o if dt == torch.bfloat16 else o.to(dt)
