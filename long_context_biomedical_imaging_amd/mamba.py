"""MambaVisionMixer — drop-in for /root/reference/model/models/mamba.py (:30-139).

Same constructor signature, parameter-creation order and state_dict keys. The forward keeps every
activation channels-last (B, L, C), the natural layout of the Linear layers, so no rearrange copies are
made: the depthwise conv + SiLU kernel reads the in_proj output in place, and the selective-scan kernel
reads u = x, delta = dt_proj(dt) and B, C as strided views of the x_proj output and writes y into the
first half of the out_proj input buffer whose second half already holds SiLU(conv(z)) — the reference's
`torch.cat([y, z], dim=1)` (mamba.py:136) without a copy.

Under bf16 autocast x_proj -> (dt, B, C) split -> dt_proj (mamba.py:120-124) run as one HIP pass per direction
(kernels.mamba_proj, lci_mamba_proj_fwd / _bwd): x_dbl never goes to HBM, dt and an aligned [B | C] tensor are
written once and the scan reads them in place; the fp32 (no-autocast) path keeps the two Linear layers.

Reference quirk kept: the dt_proj bias is applied twice (dt_proj(dt) adds it; selective_scan_fn adds it
again as delta_bias, mamba.py:120-134), so the effective delta = softplus(W dt + 2 b).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import kernels
from .blocks import TokenLinear


class MambaVisionMixer(nn.Module):
    def __init__(self, d_model, d_state=16, d_conv=4, expand=2, dt_rank="auto", dt_min=0.001, dt_max=0.1,
                 dt_init="random", dt_scale=1.0, dt_init_floor=1e-4, conv_bias=True, bias=False,
                 use_fast_path=True, layer_idx=None, device=None, dtype=None):
        factory_kwargs = {"device": device, "dtype": dtype}
        super().__init__()
        self.d_model = d_model
        self.d_state = d_state
        self.d_conv = d_conv
        self.expand = expand
        self.d_inner = int(self.expand * self.d_model)
        self.dt_rank = math.ceil(self.d_model / 16) if dt_rank == "auto" else dt_rank
        self.use_fast_path = use_fast_path
        self.layer_idx = layer_idx
        self.in_proj = TokenLinear(self.d_model, self.d_inner, bias=bias, **factory_kwargs)
        self.x_proj = TokenLinear(self.d_inner // 2, self.dt_rank + self.d_state * 2, bias=False, **factory_kwargs)
        self.dt_proj = TokenLinear(self.dt_rank, self.d_inner // 2, bias=True, **factory_kwargs)
        dt_init_std = self.dt_rank ** -0.5 * dt_scale
        if dt_init == "constant":
            nn.init.constant_(self.dt_proj.weight, dt_init_std)
        elif dt_init == "random":
            nn.init.uniform_(self.dt_proj.weight, -dt_init_std, dt_init_std)
        else:
            raise NotImplementedError
        dt = torch.exp(torch.rand(self.d_inner // 2, **factory_kwargs) * (math.log(dt_max) - math.log(dt_min))
                       + math.log(dt_min)).clamp(min=dt_init_floor)
        inv_dt = dt + torch.log(-torch.expm1(-dt))
        with torch.no_grad():
            self.dt_proj.bias.copy_(inv_dt)
        self.dt_proj.bias._no_reinit = True
        A = torch.arange(1, self.d_state + 1, dtype=torch.float32, device=device)[None, :].repeat(
            self.d_inner // 2, 1).contiguous()
        self.A_log = nn.Parameter(torch.log(A))
        self.A_log._no_weight_decay = True
        self.D = nn.Parameter(torch.ones(self.d_inner // 2, device=device))
        self.D._no_weight_decay = True
        self.out_proj = TokenLinear(self.d_inner, self.d_model, bias=bias, **factory_kwargs)
        self.conv1d_x = nn.Conv1d(in_channels=self.d_inner // 2, out_channels=self.d_inner // 2,
                                  bias=conv_bias // 2, kernel_size=d_conv, groups=self.d_inner // 2,
                                  **factory_kwargs)
        self.conv1d_z = nn.Conv1d(in_channels=self.d_inner // 2, out_channels=self.d_inner // 2,
                                  bias=conv_bias // 2, kernel_size=d_conv, groups=self.d_inner // 2,
                                  **factory_kwargs)

    def forward(self, hidden_states):
        """hidden_states (B, L, D) -> (B, L, D)."""
        xz = self.in_proj(hidden_states)                                   # (B, L, d_inner)
        # SiLU(depthwise conv 'same') of both halves; yz[..., Dx:] = SiLU(conv z), xs = SiLU(conv x)
        xs, yz = kernels.dwconv_silu_pair(xz, self.conv1d_x.weight, self.conv1d_x.bias,
                                          self.conv1d_z.weight, self.conv1d_z.bias)
        A = -torch.exp(self.A_log.float())
        N, R = self.d_state, self.dt_rank
        es = 2 if torch.is_autocast_enabled("cuda") else xs.element_size()
        Dx = self.d_inner // 2
        if kernels.mamba_proj_supported(xs, Dx, R, 2 * N) and self.dt_proj.bias is not None:
            # bf16 autocast: x_proj -> split -> dt_proj in one HIP pass (lci_mamba_proj_fwd); [B | C] as one aligned
            # (B, L, 2N) tensor the scan reads in place; the scan's u is the projection's alias of xs, so its
            # gradient is added inside the projection's backward kernel
            dt, bc, u = kernels.mamba_proj(xs, self.x_proj.weight, self.dt_proj.weight, self.dt_proj.bias, R, 2 * N,
                                           with_u=True)
            y = kernels.selective_scan_cl(u, dt, A, bc, None, self.D.float(), self.dt_proj.bias.float(), yz)
            return self.out_proj(y)
        if (R * es) % 16 or ((R + 2 * N) * es) % 16 or (N * es) % 16:
            # the scan reads B / C rows with 16-byte vectors: when dt_rank breaks their alignment (Swin stages,
            # d_model 96 / 192 -> dt_rank 6 / 12) the same projection is computed with its output columns
            # reordered to [B | C | dt | 0-pad to 8] (the weight rows permuted, gradients flow back through cat)
            pad = (-(R + 2 * N)) % 8
            W = self.x_proj.weight
            w = torch.cat([W[R:], W[:R]] + ([W.new_zeros(pad, W.shape[1])] if pad else []), 0)
            x_dbl = kernels.linear(xs, w, None)                            # (B, L, 2N + R + pad)
            Bm, Cm = x_dbl[..., :N], x_dbl[..., N:2 * N]
            dt = self.dt_proj(x_dbl[..., 2 * N:2 * N + R])
        else:
            x_dbl = self.x_proj(xs)                                        # (B, L, dt_rank + 2N)
            dt = self.dt_proj(x_dbl[..., :R])                              # (B, L, Dx), bias added once
            Bm = x_dbl[..., R: R + N]
            Cm = x_dbl[..., R + N:]
        y = kernels.selective_scan_cl(xs, dt, A, Bm, Cm, self.D.float(), self.dt_proj.bias.float(), yz)
        return self.out_proj(y)
