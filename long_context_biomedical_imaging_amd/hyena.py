"""Hyena operator — drop-in for /root/reference/model/models/hyena.py (:15-363).

Same class names, constructor signatures (pydantic `validate_call` on HyenaOperator), parameter-creation
order and state_dict keys (filter_fn.pos_emb.z / .t, filter_fn.implicit_filter.{0..6}, shared Sin freq,
filter_fn.modulation.deltas, filter_fn.bias, short_filter, in_proj, out_proj).

Forward data flow (HIP kernels in kernels.hyena_*):
  in_proj (B, L, 3D) channels-last
  -> hyena_pre: causal depthwise conv k=short_filter_order over L + pre-gate v*x1, written channel-major
     f32 for the long convolution, plus x2 (post-gate operand)
  -> implicit filter k (64, L): kernels.hyena_filter (MLP + sin + modulation fused, bf16-autocast numerics)
  -> hyena_fftconv: y = causal_conv(v*x1, k) + D (v*x1), times x2, written channels-last for out_proj.
The reference's causal long conv (fftconv_ref, n = 2L FFT) is evaluated exactly as a linear convolution
(block-partitioned FFT on the GPU), bidirectional stays False as in the reference (the `bidrectional`
kwarg is swallowed by **filter_args, backbone_vit.py:177).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
from pydantic import validate_call

from . import kernels
from .blocks import TokenLinear


class OptimModule(nn.Module):
    def register(self, name, tensor, lr=None, wd=0.0):
        if lr == 0.0:
            self.register_buffer(name, tensor)
        else:
            self.register_parameter(name, nn.Parameter(tensor))
            optim = {}
            if lr is not None:
                optim["lr"] = lr
            if wd is not None:
                optim["weight_decay"] = wd
            setattr(getattr(self, name), "_optim", optim)


class Sin(nn.Module):
    def __init__(self, dim, w=10, train_freq=True):
        super().__init__()
        self.freq = nn.Parameter(w * torch.ones(1, dim)) if train_freq else w * torch.ones(1, dim)

    def forward(self, x):
        return torch.sin(self.freq * x)


class PositionalEmbedding(OptimModule):
    def __init__(self, emb_dim: int, seq_len: int, lr_pos_emb: float = 1e-5, **kwargs):
        super().__init__()
        self.seq_len = seq_len
        t = torch.linspace(0, 1, self.seq_len)[None, :, None]
        bands = (emb_dim - 1) // 2
        t_rescaled = torch.linspace(0, seq_len - 1, seq_len)[None, :, None]
        w = 2 * math.pi * t_rescaled / seq_len
        f = torch.linspace(1e-4, bands - 1, bands)[None, None]
        z = torch.exp(-1j * f * w)
        z = torch.cat([t, z.real, z.imag], dim=-1)
        self.register("z", z, lr=lr_pos_emb)
        self.register("t", t, lr=0.0)

    def forward(self, L):
        return self.z[:, :L], self.t[:, :L]


class ExponentialModulation(OptimModule):
    def __init__(self, d_model, fast_decay_pct=0.3, slow_decay_pct=1.5, target=1e-2, modulation_lr=0.0,
                 shift: float = 0.0, **kwargs):
        super().__init__()
        self.shift = shift
        max_decay = math.log(target) / fast_decay_pct
        min_decay = math.log(target) / slow_decay_pct
        deltas = torch.linspace(min_decay, max_decay, d_model)[None, None]
        self.register("deltas", deltas, lr=modulation_lr)

    def forward(self, t, x):
        decay = torch.exp(-t * self.deltas.abs())
        return x * (decay + self.shift)


class Filter(OptimModule):
    def __init__(self, d_model, emb_dim=3, order=16, seq_len=1024, lr=1e-3, lr_pos_emb=1e-5, dropout=0.0, w=1,
                 wd=0, bias=True, num_inner_mlps=2, linear_mixer=False, modulate: bool = True,
                 normalized=False, num_heads: int = 1, **kwargs):
        super().__init__()
        self.d_model = d_model
        self.emb_dim = emb_dim
        self.seq_len = seq_len
        self.modulate = modulate
        self.num_heads = num_heads
        self.use_bias = bias
        self.bias = nn.Parameter(torch.randn(self.d_model))
        self.dropout = nn.Dropout(dropout)
        act = Sin(dim=order, w=w)
        assert emb_dim % 2 != 0 and emb_dim >= 3, \
            "emb_dim must be odd and greater or equal to 3 (time, sine and cosine)"
        self.pos_emb = PositionalEmbedding(emb_dim, seq_len, lr_pos_emb)
        if linear_mixer is False:
            layers = [nn.Linear(emb_dim, order), act]
            for _ in range(num_inner_mlps):
                layers.append(nn.Linear(order, order))
                layers.append(act)
            layers.append(nn.Linear(order, d_model, bias=False))
            self.implicit_filter = nn.Sequential(*layers)
        else:
            self.implicit_filter = nn.Sequential(nn.Linear(emb_dim, d_model, bias=False))
        self.modulation = ExponentialModulation(d_model, **kwargs)
        self.normalized = normalized
        for c in self.implicit_filter.children():
            for name, v in c.state_dict().items():
                setattr(getattr(c, name), "_optim", {"weight_decay": wd, "lr": lr})

    def filter(self, L, *args, **kwargs):
        z, t = self.pos_emb(L)
        h = self.implicit_filter(z)
        if self.modulate:
            h = self.modulation(t, h)
        if self.normalized:
            h = h / torch.norm(h, dim=-1, p=1, keepdim=True)
        return h

    def fused_filter_ok(self, L) -> bool:
        """Whether filter_k(L) runs the fused HIP implicit filter: the reference's default MLP (emb_dim <= 8,
        order = d_model = 64, num_inner_mlps = 2, one shared trainable Sin), modulation on with fixed deltas, no
        normalisation, on the GPU under bf16 autocast (LCI_FUSED_FILTER=0 turns it off)."""
        f = self.implicit_filter
        z = self.pos_emb.z
        if os.environ.get("LCI_FUSED_FILTER", "1") == "0" or not z.is_cuda:
            return False
        if not (torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16):
            return False
        if len(f) != 7 or self.d_model != 64 or not self.modulate or self.normalized or L > z.shape[1]:
            return False
        lins, acts = [f[i] for i in (0, 2, 4, 6)], [f[i] for i in (1, 3, 5)]
        if not all(isinstance(m, nn.Linear) for m in lins) or not all(a is acts[0] for a in acts):
            return False
        if not isinstance(acts[0], Sin) or not isinstance(acts[0].freq, nn.Parameter):
            return False
        shapes = [tuple(m.weight.shape) for m in lins]
        if shapes != [(64, self.emb_dim), (64, 64), (64, 64), (64, 64)] or self.emb_dim > 8:
            return False
        if lins[3].bias is not None or any(m.bias is None for m in lins[:3]):
            return False
        return isinstance(self.modulation.deltas, torch.Tensor) and \
            not isinstance(self.modulation.deltas, nn.Parameter)

    def filter_k(self, L):
        """The modulated filter as (d_model, L) = filter(L)[0].transpose(0, 1) (hyena.py:343-345)."""
        if self.fused_filter_ok(L):
            f = self.implicit_filter
            return kernels.hyena_filter(self.pos_emb.z, f[0].weight, f[0].bias, f[1].freq, f[2].weight, f[2].bias,
                                        f[4].weight, f[4].bias, f[6].weight, self.pos_emb.t, self.modulation.deltas,
                                        self.modulation.shift, L)
        return self.filter(L)[0].transpose(0, 1)

    def forward(self, x, L, k=None, bias=None, *args, **kwargs):
        """Long convolution of x (B, H, C, L) channel-major with k (C, L) plus bias*x (fftconv_ref)."""
        if k is None:
            k = self.filter_k(L)
        k = k[0] if type(k) is tuple else k
        if bias is None:
            bias = self.bias
        bias = bias if self.use_bias else 0 * bias
        return kernels.fftconv(x, k, bias.reshape(-1))


class HyenaOperator(nn.Module):
    NUM_PROJECTIONS = 3

    @validate_call
    def __init__(self, d_model: int, l_max: int, filter_order: int = 64, num_heads: int = 1, num_blocks: int = 1,
                 outer_mixing: bool = False, dropout: float = 0.0, filter_dropout: float = 0.0,
                 short_filter_order: int = 3, return_state: bool = False, bidirectional: bool = False,
                 layer_idx: int = None, **filter_args):
        super().__init__()
        assert d_model % num_heads == 0, f"Model dimension {d_model} must be divisible by num heads {num_heads}"
        assert l_max % num_blocks == 0, \
            f"Maximum signal length {l_max} must be divisible by block dimension {num_blocks}"
        if num_blocks != 1:
            raise NotImplementedError("num_blocks > 1 is not used by the reference")
        self.d_model = d_model
        self.l_max = l_max
        self.num_heads = num_heads
        self.block_dim = l_max // num_blocks
        self.head_dim = d_model // num_heads
        self.filter_order = filter_order
        self.short_filter_order = short_filter_order
        self.num_blocks = num_blocks
        self.filter_dropout = filter_dropout
        self.outer_mixing = outer_mixing
        self.return_state = return_state
        self.dropout = nn.Dropout(dropout)
        self.in_proj = TokenLinear(self.d_model, self.NUM_PROJECTIONS * self.d_model)
        self.out_proj = TokenLinear(self.d_model, self.d_model)
        self.bidirectional = bidirectional
        total_width = self.d_model * self.NUM_PROJECTIONS
        self.short_filter = nn.Conv1d(in_channels=total_width, out_channels=total_width,
                                      kernel_size=self.short_filter_order, groups=total_width,
                                      padding=self.short_filter_order - 1)
        if "channels" not in filter_args:
            filter_args["channels"] = 1
        self.filter_fn = Filter(self.head_dim, order=self.filter_order, seq_len=self.l_max,
                                dropout=self.filter_dropout, bidirectional=self.bidirectional, l_max=self.l_max,
                                **filter_args)

    def forward(self, u, *args, **kwargs):
        """u (B, L, D) -> (B, L, D)."""
        l = u.size(1)
        if l > self.l_max:
            # the reference's assert message names a missing attribute (hyena.py:314) -> AttributeError
            raise AttributeError(f"Input length {l} exceeds maximum length {self.l_max} "
                                 "('HyenaOperator' object has no attribute 'max_l' in the reference)")
        if self.bidirectional:
            raise NotImplementedError("bidirectional Hyena is never enabled by the reference")
        if self.training and self.dropout.p > 0:
            raise NotImplementedError("Hyena dropout > 0 is not fused")
        z = self.in_proj(u)                                                    # (B, L, 3D)
        v, x2 = kernels.hyena_pre(z, self.short_filter.weight, self.short_filter.bias, self.num_heads)
        k = self.filter_fn.filter_k(l)                                         # (head_dim, L)
        bias = self.filter_fn.bias if self.filter_fn.use_bias else 0 * self.filter_fn.bias
        y = kernels.hyena_fftconv_gate(v, k, bias, x2)                         # (B, L, D) channels-last
        y = self.out_proj(y)
        if self.return_state:
            return y, None
        return y

    def state_size(self, sequence_length: int = 2048) -> int:
        return self.d_model * sequence_length
