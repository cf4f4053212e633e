"""Function-level drop-ins with the exact signatures the reference calls.

  selective_scan_fn   mamba-ssm 1.2.0.post1 `mamba_ssm.ops.selective_scan_interface.selective_scan_fn`,
                      called at /root/reference/model/models/mamba.py:125-134 (channel-major (B, D, L) tensors)
  fftconv_ref         /root/reference/model/models/hyena.py:32-51

Both run the liblci HIP kernels. selective_scan_fn transposes the channel-major operands to the kernel's
channels-last layout (the module-level MambaVisionMixer avoids those copies by keeping everything
channels-last end to end).
"""
from __future__ import annotations

import torch

from . import kernels


def selective_scan_fn(u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False,
                      return_last_state=False):
    """u, delta (b, d, L); A (d, n) real; B, C (b, n, L) ('variable B/C'); D, delta_bias (d). Output in u.dtype."""
    if z is not None:
        raise NotImplementedError("z-gating is never used by the reference (mamba.py:493 passes z=None)")
    if A.is_complex() or B.dim() != 3 or C.dim() != 3:
        raise NotImplementedError("only real A with (b, n, L) B/C, as called by the reference")
    b, d, L = u.shape
    n = A.shape[1]
    dt = u.dtype if u.dtype in (torch.bfloat16, torch.float32) else torch.float32
    ucl = u.to(dt).transpose(1, 2).contiguous()
    dcl = delta.to(dt).transpose(1, 2).contiguous()
    bc = torch.cat([B.to(dt).transpose(1, 2), C.to(dt).transpose(1, 2)], dim=-1).contiguous()
    yz = torch.empty(b, L, 2 * d, device=u.device, dtype=dt)
    res = kernels.selective_scan_cl(ucl, dcl, A, bc[..., :n], bc[..., n:], D, delta_bias, yz,
                                    delta_softplus=delta_softplus, return_last_state=return_last_state)
    out, last = res if return_last_state else (res, None)
    y = out[..., :d].transpose(1, 2).to(u.dtype)
    return (y, last) if return_last_state else y


def fftconv_ref(u, k, D, dropout_mask, gelu=True, k_rev=None):
    """Causal long conv (n = 2L FFT semantics) + D u; u (b, H, C, 1, L) or (b, C, L); k (C, L)."""
    if k_rev is not None:
        raise NotImplementedError("bidirectional (k_rev) is never enabled by the reference")
    shp = u.shape
    L = shp[-1]
    C = k.shape[0]
    Dv = D.reshape(-1)
    rows = u.reshape(-1, C, L) if u.dim() <= 3 else u.reshape(shp[0], shp[1], C, L)
    y = kernels.fftconv(rows, k, Dv).reshape(shp)
    if gelu:
        y = torch.nn.functional.gelu(y)
    if dropout_mask is not None:
        y = y * dropout_mask.reshape(*dropout_mask.shape, *([1] * (y.dim() - dropout_mask.dim())))
    return y.to(u.dtype)
