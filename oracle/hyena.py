"""Oracle: Hyena operator, CPU restatement. Test infrastructure only.

Follows /root/reference/model/models/hyena.py:
  :32-51    fftconv_ref: y = irfft(rfft(u, 2L) * rfft(k, 2L)/2L, norm="forward")[:L] + u*D  (gelu=False)
  :67-89    PositionalEmbedding z = [t, cos(f w), -sin(f w)], t = linspace(0,1,l_max)
  :54-64    Sin (one shared freq Parameter per Filter)
  :92-113   ExponentialModulation h *= exp(-t |deltas|)
  :190-199  Filter.filter
  :306-360  HyenaOperator.forward (in_proj -> causal dwconv k -> x1,x2,v -> v*x1 -> long conv -> *x2)
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def pos_emb(l_max: int, emb_dim: int = 3):
    """PositionalEmbedding buffers (hyena.py:68-86): returns z (1, l_max, emb_dim), t (1, l_max, 1)."""
    t = torch.linspace(0, 1, l_max)[None, :, None]
    bands = (emb_dim - 1) // 2
    t_rescaled = torch.linspace(0, l_max - 1, l_max)[None, :, None]
    w = 2 * math.pi * t_rescaled / l_max
    f = torch.linspace(1e-4, bands - 1, bands)[None, None]
    z = torch.exp(-1j * f * w)
    z = torch.cat([t, z.real, z.imag], dim=-1)
    return z, t


def deltas(d_model: int, fast_decay_pct=0.3, slow_decay_pct=1.5, target=1e-2):
    """ExponentialModulation.deltas (hyena.py:103-107)."""
    max_decay = math.log(target) / fast_decay_pct
    min_decay = math.log(target) / slow_decay_pct
    return torch.linspace(min_decay, max_decay, d_model)[None, None]


def implicit_filter(L, z, t, lin_ws, lin_bs, freq, dlt, shift=0.0):
    """Filter.filter (hyena.py:190-199): MLP with shared Sin, then exp-decay modulation -> (1, L, d)."""
    h = z[:, :L]
    n = len(lin_ws)
    for i, (w, b) in enumerate(zip(lin_ws, lin_bs)):
        h = F.linear(h, w, b)
        if i < n - 1:
            h = torch.sin(freq * h)
    decay = torch.exp(-t[:, :L] * dlt.abs())
    return h * (decay + shift)


def fftconv(u, k, D):
    """fftconv_ref with gelu=False, no dropout (hyena.py:32-51). u (..., C, L); k (C, L); D (C,).

    (The reference carries a singleton block axis, u (b, h, C, 1, L), and unsqueezes k_f to match;
    here that axis is squeezed, so k_f broadcasts over the leading axes directly.)
    """
    L = u.shape[-1]
    n = 2 * L
    k_f = torch.fft.rfft(k, n=n) / n
    u_f = torch.fft.rfft(u.to(k.dtype), n=n)
    y = torch.fft.irfft(u_f * k_f, n=n, norm="forward")[..., :L]
    return (y + u * D.unsqueeze(-1)).to(u.dtype)


def causal_conv_direct(u, k, D):
    """Same result as fftconv by direct summation (float64; small L only): y[t]=sum_{s<=t} k[t-s]u[s]+D u[t]."""
    L = u.shape[-1]
    uu = u.double()
    kk = k.double()
    y = torch.zeros_like(uu)
    for t in range(L):
        y[..., t] = (uu[..., : t + 1] * kk[..., : t + 1].flip(-1)).sum(-1)
    return y + uu * D.double().unsqueeze(-1)


def short_conv(u, weight, bias, L):
    """Depthwise Conv1d(groups=C, k, padding=k-1) then keep first L (hyena.py:285-291, :321)."""
    kk = weight.shape[-1]
    return F.conv1d(u, weight, bias, padding=kk - 1, groups=u.shape[1])[..., :L]


def hyena_forward(u, p, num_heads, l_max=66000):
    """HyenaOperator.forward (hyena.py:306-360) with num_blocks=1, bidirectional=False.

    p: dict with in_proj.{weight,bias}, out_proj.{weight,bias}, short_filter.{weight,bias},
       filter_fn.bias, filter_fn.implicit_filter.{0,2,4,6}.weight (+.bias for 0,2,4), freq, z, t, deltas.
    """
    b, L, d = u.shape
    if L > l_max:
        raise AssertionError(f"Input length {L} exceeds maximum length {l_max}")
    x = F.linear(u, p["in_proj.weight"], p["in_proj.bias"]).transpose(1, 2)
    uc = short_conv(x, p["short_filter.weight"], p["short_filter.bias"], L)
    hd = d // num_heads
    uc = uc.reshape(b, num_heads, 3 * hd, L)
    x1, x2, v = uc.split(hd, dim=2)
    v = v * x1
    ws = [p[f"filter_fn.implicit_filter.{i}.weight"] for i in (0, 2, 4, 6)]
    bs = [p.get(f"filter_fn.implicit_filter.{i}.bias") for i in (0, 2, 4, 6)]
    k = implicit_filter(L, p["filter_fn.pos_emb.z"], p["filter_fn.pos_emb.t"], ws, bs,
                        p["filter_fn.implicit_filter.1.freq"], p["filter_fn.modulation.deltas"])
    k = k[0].transpose(0, 1)  # (hd, L)
    v = fftconv(v, k, p["filter_fn.bias"])
    v = v * x2
    y = v.reshape(b, d, L).transpose(1, 2)
    return F.linear(y, p["out_proj.weight"], p["out_proj.bias"])
