"""GPU parity: selective scan / depthwise conv+SiLU / MambaVisionMixer (liblci) vs the reference's outputs.

fp32 I/O: the scan is f32 arithmetic like mamba-ssm's kernel; tolerance rel L2 <= 1e-4 (exp2/log1p
hardware approximations and summation order). bf16 I/O (autocast): rel L2 <= 2e-2.
"""
import pytest
import torch
import torch.nn.functional as F

from golden_util import Golden, cotangents, rel_err
from oracle import selective_scan as oscan

pytestmark = pytest.mark.gpu


def _cl(t):  # (b, c, L) -> (b, L, c)
    return t.transpose(1, 2).contiguous()


def _run_scan(u, delta, A, Bm, Cm, D, db, cot, dtype=torch.float32):
    from long_context_biomedical_imaging_amd import kernels
    b, d, L = u.shape
    N = A.shape[1]
    dev = "cuda"
    uc = _cl(u).to(dev, dtype).requires_grad_(True)
    dc = _cl(delta).to(dev, dtype).requires_grad_(True)
    Ac = A.to(dev).requires_grad_(True)
    x_dbl = torch.cat([_cl(Bm), _cl(Cm)], dim=-1).to(dev, dtype).requires_grad_(True)
    Dc = D.to(dev).requires_grad_(True)
    bc = db.to(dev).requires_grad_(True)
    yz = torch.zeros(b, L, 2 * d, device=dev, dtype=dtype)
    out = kernels.selective_scan_cl(uc, dc, Ac, x_dbl[..., :N], x_dbl[..., N:], Dc, bc, yz)
    y = out[..., :d]
    (y.float() * _cl(cot).to(dev)).sum().backward()
    grads = {"u": uc.grad.transpose(1, 2), "delta": dc.grad.transpose(1, 2), "A": Ac.grad,
             "B": x_dbl.grad[..., :N].transpose(1, 2), "C": x_dbl.grad[..., N:].transpose(1, 2), "D": Dc.grad,
             "delta_bias": bc.grad}
    return y.transpose(1, 2).detach(), grads


def test_selective_scan_vs_reference_fixture():
    g = Golden("selective_scan")
    names = ["u", "delta", "A", "B", "C", "D", "delta_bias"]
    ins = [g.t(f"in/{n}") for n in names]
    y, grads = _run_scan(*ins, g.t("cot/y"))
    assert rel_err(y, g.t("out/y")) < 1e-4
    for n in names:
        assert rel_err(grads[n], g.t(f"grad/{n}")) < 2e-4, n


@pytest.mark.parametrize("L,d,dtype,tol", [(5000, 96, torch.float32, 2e-4), (3001, 64, torch.bfloat16, 3e-2)])
def test_selective_scan_chunked_long(L, d, dtype, tol):
    """Many chunks (chunk 256): the cross-chunk carries (fwd and bwd) are exercised; ragged tail."""
    torch.manual_seed(3)
    b, n = 1, 8
    u = torch.randn(b, d, L)
    delta = torch.randn(b, d, L) * 0.5 - 1.0
    A = -torch.exp(torch.randn(d, n) * 0.3)
    Bm, Cm = torch.randn(b, n, L), torch.randn(b, n, L)
    D, db = torch.randn(d), torch.randn(d) * 0.1
    cot = torch.randn(b, d, L)
    y, grads = _run_scan(u, delta, A, Bm, Cm, D, db, cot, dtype)
    q = lambda t: t.to(dtype).float()  # noqa: E731  (reference sees the same rounded inputs)
    ins = [q(u).double().requires_grad_(True), q(delta).double().requires_grad_(True), A.double().requires_grad_(True),
           q(Bm).double().requires_grad_(True), q(Cm).double().requires_grad_(True), D.double().requires_grad_(True),
           db.double().requires_grad_(True)]
    yr = oscan.selective_scan(*ins[:6], delta_bias=ins[6], delta_softplus=True, chunk=1024)
    (yr * cot.double()).sum().backward()
    assert rel_err(y, yr) < tol
    for name, r in zip(["u", "delta", "A", "B", "C", "D", "delta_bias"], ins):
        assert rel_err(grads[name], r.grad) < 5 * tol, name


@pytest.mark.parametrize("dtype,L,C,bias", [(torch.float32, 700, 96, False), (torch.float32, 257, 96, True),
                                             (torch.bfloat16, 1000, 192, True), (torch.bfloat16, 513, 36, False)])
def test_dwconv_silu_pair(dtype, L, C, bias):
    """mamba.py:118-119 conv1d(k=3, 'same', groups=C) + SiLU on both halves: vector forward when C % V == 0 (V = 4 f32 /
    8 bf16; C=36 bf16 takes the scalar forward), 4-channel vector backward; runs across the 256-token boundary."""
    from long_context_biomedical_imaging_amd import kernels
    torch.manual_seed(0)
    B = 2
    xz = torch.randn(B, L, 2 * C).to(dtype).float()
    wx, wz = torch.randn(C, 1, 3), torch.randn(C, 1, 3)
    bx, bz = (torch.randn(C), torch.randn(C)) if bias else (None, None)
    x = xz.to(dtype).cuda().requires_grad_(True)
    wxc, wzc = wx.cuda().requires_grad_(True), wz.cuda().requires_grad_(True)
    bxc, bzc = (bx.cuda().requires_grad_(True), bz.cuda().requires_grad_(True)) if bias else (None, None)
    xs, yz = kernels.dwconv_silu_pair(x, wxc, bxc, wzc, bzc)
    xr = xz.clone().requires_grad_(True)
    wxr, wzr = wx.clone().requires_grad_(True), wz.clone().requires_grad_(True)
    bxr, bzr = (bx.clone().requires_grad_(True), bz.clone().requires_grad_(True)) if bias else (None, None)
    xx, zz = xr.transpose(1, 2).chunk(2, dim=1)
    rx = F.silu(F.conv1d(xx, wxr, bxr, padding="same", groups=C)).transpose(1, 2)
    rz = F.silu(F.conv1d(zz, wzr, bzr, padding="same", groups=C)).transpose(1, 2)
    tol = 1e-5 if dtype == torch.float32 else 8e-3   # bf16 outputs: one rounding (2^-9 relative)
    assert rel_err(xs.float(), rx) < tol and rel_err(yz[..., C:].float(), rz) < tol
    cx, cz = torch.randn(B, L, C).to(dtype).float(), torch.randn(B, L, C).to(dtype).float()
    gyz = torch.cat([torch.zeros(B, L, C), cz], -1)
    torch.autograd.backward([xs, yz], [cx.to(dtype).cuda(), gyz.to(dtype).cuda()])
    torch.autograd.backward([rx, rz], [cx, cz])
    assert rel_err(x.grad.float(), xr.grad) < tol
    assert rel_err(wxc.grad, wxr.grad) < 10 * tol and rel_err(wzc.grad, wzr.grad) < 10 * tol
    if bias:
        assert rel_err(bxc.grad, bxr.grad) < 10 * tol and rel_err(bzc.grad, bzr.grad) < 10 * tol


@pytest.mark.parametrize("amp", [False, True])
def test_mamba_mixer_vs_reference(amp):
    from long_context_biomedical_imaging_amd import mamba
    g = Golden("mamba_mixer")
    m = mamba.MambaVisionMixer(d_model=128, d_state=8, d_conv=3, expand=1)
    m.load_state_dict(g.sd())
    m = m.cuda()
    x = g.t("in/x").cuda().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        out = m(x)
    tol = 2e-2 if amp else 1e-4
    assert rel_err(out, g.t("out/0")) < tol
    out.float().backward(cotangents([out])[0].cuda())
    assert rel_err(x.grad, g.t("grad/in0")) < (5e-2 if amp else 2e-4)
    for p in ("A_log", "D", "dt_proj.bias", "x_proj.weight", "in_proj.weight", "conv1d_x.weight"):
        assert rel_err(dict(m.named_parameters())[p].grad, g.t(f"grad/{p}")) < (6e-2 if amp else 3e-4), p


def test_compat_selective_scan_fn_signature():
    """mamba-ssm selective_scan_fn signature (channel-major) vs the reference fixture; last state vs oracle loop."""
    from long_context_biomedical_imaging_amd.compat import selective_scan_fn
    g = Golden("selective_scan")
    names = ["u", "delta", "A", "B", "C", "D", "delta_bias"]
    ins = {n: g.t(f"in/{n}").cuda() for n in names}
    y, last = selective_scan_fn(ins["u"], ins["delta"], ins["A"], ins["B"], ins["C"], ins["D"], z=None,
                                delta_bias=ins["delta_bias"], delta_softplus=True, return_last_state=True)
    assert rel_err(y, g.t("out/y")) < 1e-4
    u, dl, A, Bm = (g.t(f"in/{n}").double() for n in ("u", "delta", "A", "B"))
    dt = F.softplus(dl + g.t("in/delta_bias").double()[:, None])
    x = torch.zeros(u.shape[0], u.shape[1], A.shape[1], dtype=torch.float64)
    for t in range(u.shape[2]):
        x = torch.exp(dt[:, :, t, None] * A[None]) * x + (dt[:, :, t] * u[:, :, t])[..., None] * Bm[:, None, :, t]
    assert rel_err(last, x) < 1e-4
    dpos = g.t("in/delta").abs() * 0.2 + 0.01   # positive dt without softplus (a stable recurrence)
    y2 = selective_scan_fn(ins["u"], dpos.cuda(), ins["A"], ins["B"], ins["C"], ins["D"], delta_bias=None,
                           delta_softplus=False)
    t6 = [g.t(f"in/{n}").double() for n in names[:6]]
    t6[1] = dpos.double()
    yr = oscan.selective_scan(*t6, delta_bias=None, delta_softplus=False)
    assert rel_err(y2, yr) < 1e-4


@pytest.mark.parametrize("d_model,B,L", [(384, 1, 4096), (96, 64, 64), (128, 2, 777), (768, 2, 512)])
def test_fused_mamba_projection_matches_linear_layers(d_model, B, L, monkeypatch):
    """lci_mamba_proj (x_proj -> split -> dt_proj fused, mamba.py:120-124) against the two torch Linear layers it
    replaces, both under bf16 autocast: output and every parameter / input gradient within rel-L2 1e-2 (bf16
    intermediates rounded at the same points, f32 accumulation in a different order). Shapes: ViT (Dx 192, dt_rank
    24), Swin stage 1 windows (Dx 48, dt_rank 6), the golden's d_model 128, Swin stage 4 (Dx 384, dt_rank 48)."""
    from long_context_biomedical_imaging_amd import kernels, mamba
    torch.manual_seed(d_model + L)
    m = mamba.MambaVisionMixer(d_model=d_model, d_state=8, d_conv=3, expand=1).cuda()
    x = torch.randn(B, L, d_model, device="cuda")
    cot = torch.randn(B, L, d_model, device="cuda")
    res = {}
    for fused in (True, False):
        monkeypatch.setenv("LCI_MAMBA_PROJ", "1" if fused else "0")
        m.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if fused:
                xs_probe = torch.zeros(B, L, d_model // 2, device="cuda", dtype=torch.bfloat16)
                assert kernels.mamba_proj_supported(xs_probe, d_model // 2, m.dt_rank, 16)
            out = m(xi)
        out.float().backward(cot)
        res[fused] = {"out": out.detach().float(), "x": xi.grad.detach().clone(),
                      **{n: p.grad.detach().clone() for n, p in m.named_parameters()}}
    for k, ref in res[False].items():
        assert rel_err(res[True][k], ref) < 1e-2, (k, rel_err(res[True][k], ref))


@pytest.mark.parametrize("nseq,L,d,dtype", [(300, 64, 48, torch.bfloat16), (40, 343, 96, torch.float32),
                                           (8, 512, 384, torch.bfloat16), (3, 37, 200, torch.float32)])
def test_selective_scan_one_chunk_path_bitwise(nseq, L, d, dtype):
    """Window sequences (one chunk, ABI 32): without a requested final state the forward runs only the output pass
    and the backward skips the adjoint aggregate / carry, and dB / dC are stored rather than accumulated where one
    workgroup holds every channel (Dx <= 256). Nothing is carried into a single chunk, so y, du and d(delta) must
    equal the full three-pass path (forced by return_last_state=True) bit for bit. dB / dC are summed over the
    workgroup's waves with LDS float atomics, and dA / dD / d(delta_bias) over per-(b, chunk) partials with float
    atomics, in either path: their summation order varies from run to run, so they match to f32 rounding."""
    from long_context_biomedical_imaging_amd import kernels
    torch.manual_seed(nseq + L)
    n = 8
    dev = "cuda"
    u = torch.randn(nseq, L, d, device=dev).to(dtype)
    delta = (torch.randn(nseq, L, d, device=dev) * 0.5 - 1.0).to(dtype)
    A = -torch.exp(torch.randn(d, n, device=dev) * 0.3)
    bc = torch.randn(nseq, L, 2 * n, device=dev).to(dtype)
    D, db = torch.randn(d, device=dev), torch.randn(d, device=dev) * 0.1
    cot = torch.randn(nseq, L, d, device=dev)
    res = []
    for want_last in (False, True):
        leaves = [t.detach().clone().requires_grad_(True) for t in (u, delta, A, bc, D, db)]
        uc, dc, Ac, bcc, Dc, dbc = leaves
        yz = torch.zeros(nseq, L, 2 * d, device=dev, dtype=dtype)
        out = kernels.selective_scan_cl(uc, dc, Ac, bcc[..., :n], bcc[..., n:], Dc, dbc, yz,
                                        return_last_state=want_last)
        if want_last:
            out, last = out
            assert last.shape == (nseq, d, n) and torch.isfinite(last).all()
        (out[..., :d].float() * cot).sum().backward()
        res.append([out[..., :d].detach()] + [t.grad for t in leaves])
    names = ("y", "du", "ddelta", "dA", "dBC", "dD", "ddelta_bias")
    for name, a, b in zip(names, *res):
        if name in ("dA", "dBC", "dD", "ddelta_bias"):   # summed by float atomics: the order varies
            # (f32 sums to f32 rounding; in a bf16 gradient tensor that can flip the output's last bit)
            ulp = 2.0 ** -7 if a.dtype == torch.bfloat16 else 0.0
            err = ((a.float() - b.float()).abs() - ulp * b.float().abs()).max().item()
            assert err <= 1e-4 * b.float().abs().max().item() + 1e-6, (name, err)
        else:
            assert torch.equal(a, b), name
