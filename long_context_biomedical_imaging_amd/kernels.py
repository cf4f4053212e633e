"""torch.autograd wrappers over the liblci C-ABI. Each op runs the HIP kernels; none has a CPU path."""
from __future__ import annotations

import torch

from . import _lib


class KernelTimer:
    """Optional HIP-event timing of individual liblci launches, recorded on the launch stream.

    bench.py enables it for the timed region; each entry is (name, start_event, end_event, algorithmic work).
    """
    enabled = False
    records: list = []

    @classmethod
    def run(cls, name, work, t, fn):
        if not cls.enabled:
            fn()
            return
        st = torch.cuda.current_stream(t.device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn()
        e1.record(st)
        cls.records.append((name, e0, e1, work))

    @classmethod
    def summary(cls):
        """name -> {calls, avg_ms, total_ms, work_per_call} (synchronizes)."""
        torch.cuda.synchronize()
        out = {}
        for name, e0, e1, work in cls.records:
            d = out.setdefault(name, {"calls": 0, "total_ms": 0.0, "work_per_call": work})
            d["calls"] += 1
            d["total_ms"] += e0.elapsed_time(e1)
        for d in out.values():
            d["avg_ms"] = d["total_ms"] / d["calls"]
        return out

    @classmethod
    def reset(cls):
        cls.records = []


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
    KernelTimer.run("attn_fwd", 4.0 * B * num_heads * L * L * dh, qkv, lambda: _lib.call(
        "lci_attn_fwd", qkv.data_ptr(), out.data_ptr(), lse2.data_ptr(), B, L, num_heads, dh, float(scale),
        _lib.stream_of(qkv)))
    return out, lse2


def attn_bwd(qkv, out, dout, lse2, num_heads: int, scale: float):
    _lib.require_gpu(qkv, out, dout, lse2)
    B, L, C = qkv.shape
    dh = C // (3 * num_heads)
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B, num_heads, L, device=qkv.device, dtype=torch.float32)
    args = (qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse2.data_ptr(), dqkv.data_ptr(), delta.data_ptr(),
            B, L, num_heads, dh, float(scale), _lib.stream_of(qkv))
    if not KernelTimer.enabled:
        _lib.call("lci_attn_bwd", *args)
        return dqkv
    f = float(B) * num_heads * L * L * dh
    # same three launches as lci_attn_bwd, timed one by one (algorithmic FLOPs: dP, dV, dK | dQ)
    KernelTimer.run("attn_bwd_delta", 0.0, qkv, lambda: _lib.call("lci_attn_bwd_stage", 0, *args))
    KernelTimer.run("attn_bwd_dkdv", 6.0 * f, qkv, lambda: _lib.call("lci_attn_bwd_stage", 1, *args))
    KernelTimer.run("attn_bwd_dq", 2.0 * f, qkv, lambda: _lib.call("lci_attn_bwd_stage", 2, *args))
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


# ------------------------------------------------------------------------------------- patch embed
_DT = {torch.float32: 0, torch.bfloat16: 1}


def _i32arr(vals):
    import ctypes
    return (ctypes.c_int * 3)(*(list(vals) + [1] * (3 - len(vals))))


class _PatchEmbed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, pos, channels_last, out_dtype):
        B, C = x.shape[:2]
        S = list(x.shape[2:])
        D = w.shape[0]
        P = list(w.shape[2:])
        G = [-(-s // p) for s, p in zip(S, P)]
        L = 1
        for g in G:
            L *= g
        y = torch.empty((B, L, D) if channels_last else (B, D, *G), device=x.device, dtype=out_dtype)
        wf = w.float().contiguous()
        bf = bias.float().contiguous() if bias is not None else None
        pf = pos.float().reshape(L, D).contiguous() if pos is not None else None
        _lib.call("lci_patch_embed_fwd", x.data_ptr(), _DT[x.dtype], wf.data_ptr(), _lib.ptr(bf), _lib.ptr(pf),
                  y.data_ptr(), _DT[out_dtype], B, C, D, len(S), _i32arr(S), _i32arr(P), int(channels_last),
                  _lib.stream_of(x))
        ctx.save_for_backward(x)
        ctx.meta = (B, C, D, S, P, L, channels_last, w.shape, w.dtype, bias is not None, pos is not None,
                    pos.shape if pos is not None else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        B, C, D, S, P, L, cl, wshape, wdtype, has_b, has_p, pshape = ctx.meta
        dy = dy.contiguous()
        if dy.dtype not in _DT:
            dy = dy.float()
        dw = torch.zeros(wshape, device=x.device, dtype=torch.float32)
        db = torch.zeros(D, device=x.device, dtype=torch.float32) if has_b else None
        dpos = torch.empty(pshape, device=x.device, dtype=torch.float32) if has_p else None
        _lib.call("lci_patch_embed_bwd", x.data_ptr(), _DT[x.dtype], dy.data_ptr(), _DT[dy.dtype], dw.data_ptr(),
                  _lib.ptr(db), _lib.ptr(dpos), B, C, D, len(S), _i32arr(S), _i32arr(P), int(cl),
                  _lib.stream_of(x))
        if ctx.needs_input_grad[0]:
            raise NotImplementedError("patch_embed: gradient w.r.t. the input image is not provided")
        return None, dw.to(wdtype), (db if has_b else None), dpos, None, None


def patch_embed(x, weight, bias, pos, channels_last_tokens: bool):
    """Conv(k = s = patch) + bias (+ pos) via the HIP kernel.

    channels_last_tokens=True (ViT PatchEmbeddingBlock): (B, C, *S) -> (B, L, D) in f32 (the reference's
    bf16-conv + f32 pos-embed add promotes to f32). False (Swin PatchEmbed): (B, C, *S) -> (B, D, *ceil(S/p))
    in the autocast dtype when autocast is on (the reference's conv output dtype), else f32.
    """
    _lib.require_gpu(x.contiguous())
    x = x.contiguous()
    if x.dtype not in _DT:
        x = x.float()
    if channels_last_tokens:
        out_dtype = torch.float32
    else:
        out_dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else torch.float32
        if out_dtype not in _DT:
            out_dtype = torch.float32
    return _PatchEmbed.apply(x, weight, bias, pos, channels_last_tokens, out_dtype)
