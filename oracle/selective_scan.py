"""Oracle: Mamba selective scan + MambaVisionMixer, CPU restatement. Test infrastructure only.

selective_scan: third-party mamba-ssm==1.2.0.post1 (README.md:15), `selective_scan_fn` called at
/root/reference/model/models/mamba.py:125-134 (file lines 487-496 of the concatenated listing: the
call `selective_scan_fn(x, dt, A, B, C, self.D.float(), z=None, delta_bias=self.dt_proj.bias.float(),
delta_softplus=True, return_last_state=None)`). Restates the published `selective_scan_ref`:
    delta' = softplus(delta + delta_bias)          (threshold 20, torch semantics)
    x_t    = exp(delta'_t A) * x_{t-1} + delta'_t B_t u_t        per (b, d, n)
    y_t    = sum_n C_t[n] x_t[n] + D u_t
with fp32 math and output cast to u.dtype.

mamba_mixer: MambaVisionMixer.forward (mamba.py:108-139), including the reference quirk that the
dt_proj bias is added twice (once by dt_proj, once as delta_bias).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def selective_scan(u, delta, A, B, C, D=None, delta_bias=None, delta_softplus=True, chunk=None):
    """u, delta (b, d, L); A (d, n); B, C (b, n, L); D, delta_bias (d,). Returns y (b, d, L) in u.dtype.

    chunk: evaluate the recurrence chunk-by-chunk (same arithmetic order per step; only bounds the
    size of the exp(delta A) temporaries at large L).
    """
    dtype_in = u.dtype
    ct = torch.promote_types(u.dtype, torch.float32)   # f32 math as mamba-ssm; f64 inputs stay f64 (gradcheck)
    u = u.to(ct)
    delta = delta.to(ct)
    if delta_bias is not None:
        delta = delta + delta_bias[..., None].to(ct)
    if delta_softplus:
        delta = F.softplus(delta)
    b, d, L = u.shape
    A = A.to(ct)
    B = B.to(ct)
    C = C.to(ct)
    x = A.new_zeros((b, d, A.shape[1]))
    chunk = chunk or L
    ys = []
    for s in range(0, L, chunk):
        e = min(L, s + chunk)
        dA = torch.exp(torch.einsum("bdl,dn->bdln", delta[..., s:e], A))
        dBu = torch.einsum("bdl,bnl,bdl->bdln", delta[..., s:e], B[..., s:e], u[..., s:e])
        for i in range(e - s):
            x = dA[:, :, i] * x + dBu[:, :, i]
            ys.append(torch.einsum("bdn,bn->bd", x, C[:, :, s + i]))
    y = torch.stack(ys, dim=2)
    if D is not None:
        y = y + u * D[:, None].to(ct)
    return y.to(dtype_in)


def mamba_mixer(h, p, d_state=8, d_conv=3):
    """MambaVisionMixer.forward (mamba.py:108-139). p: state_dict-keyed tensors."""
    b, L, _ = h.shape
    xz = F.linear(h, p["in_proj.weight"], p.get("in_proj.bias")).transpose(1, 2)
    x, z = xz.chunk(2, dim=1)
    di = x.shape[1]
    A = -torch.exp(p["A_log"].float())
    x = F.silu(F.conv1d(x, p["conv1d_x.weight"], p.get("conv1d_x.bias"), padding="same", groups=di))
    z = F.silu(F.conv1d(z, p["conv1d_z.weight"], p.get("conv1d_z.bias"), padding="same", groups=di))
    x_dbl = F.linear(x.transpose(1, 2).reshape(b * L, di), p["x_proj.weight"])
    dt_rank = p["dt_proj.weight"].shape[1]
    dt, Bm, Cm = torch.split(x_dbl, [dt_rank, d_state, d_state], dim=-1)
    dt = F.linear(dt, p["dt_proj.weight"], p["dt_proj.bias"]).reshape(b, L, di).transpose(1, 2)
    Bm = Bm.reshape(b, L, d_state).transpose(1, 2).contiguous()
    Cm = Cm.reshape(b, L, d_state).transpose(1, 2).contiguous()
    y = selective_scan(x, dt, A, Bm, Cm, p["D"].float(), p["dt_proj.bias"].float(), True)
    y = torch.cat([y, z], dim=1).transpose(1, 2)
    return F.linear(y, p["out_proj.weight"], p.get("out_proj.bias"))


def scan_bytes_per_token(dim=192, d_state=8, s=2, bwd=False):
    """Algorithmic HBM bytes per token: fwd s(3D+2N), bwd adds s(2D+2N)."""
    fwd = s * (3 * dim + 2 * d_state)
    return fwd + (s * (2 * dim + 2 * d_state) if bwd else 0)
