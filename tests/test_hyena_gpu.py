"""GPU parity: Hyena long convolution and operator (liblci) vs the reference / oracle.

The long conv runs in f32 like the reference (u cast to k's f32 for torch.fft): tolerance rel L2 <= 2e-5
against the reference's fftconv_ref outputs, <= 1e-4 for gradients vs f64 autograd of the oracle.
Module level under bf16 autocast: outputs <= 2e-2, gradients <= 5e-2.
"""
import pytest
import torch

from golden_util import Golden, cotangents, rel_err
from oracle import hyena as oh

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("L", [1000, 2048])
def test_fftconv_vs_reference_vectors(L):
    from long_context_biomedical_imaging_amd import kernels
    g = Golden(f"fftconv_L{L}")
    u, k, D = g.t("in/u"), g.t("in/k"), g.t("in/D")
    uc, kc, Dc = (t.cuda().requires_grad_(True) for t in (u, k, D))
    y = kernels.fftconv(uc, kc, Dc)
    assert rel_err(y, g.t("out/y")) < 2e-5
    cot = torch.randn(y.shape)
    y.backward(cot.cuda())
    ur, kr, Dr = (t.double().requires_grad_(True) for t in (u, k, D))
    (oh.fftconv(ur, kr, Dr) * cot.double()).sum().backward()
    assert rel_err(uc.grad, ur.grad) < 1e-4
    assert rel_err(kc.grad, kr.grad) < 1e-4
    assert rel_err(Dc.grad, Dr.grad) < 1e-4


@pytest.mark.parametrize("R,C,L", [(3, 32, 343), (2, 8, 4096), (1, 4, 65536), (5, 3, 777), (3, 2, 100000)])
def test_fftconv_shapes(R, C, L):
    """Odd row counts (a half-empty pair), non-power-of-two L (Swin windows 7^3 = 343), the metric L, and n = 2^18
    (n1 = 512 column FFTs)."""
    from long_context_biomedical_imaging_amd import kernels
    torch.manual_seed(R * 1000 + L)
    u = torch.randn(R, C, L)
    k = torch.randn(C, L) * torch.exp(-torch.linspace(0, 8, L))[None]
    D = torch.randn(C)
    y = kernels.fftconv(u.cuda(), k.cuda(), D.cuda())
    ref = oh.fftconv(u.double(), k.double(), D.double())
    assert rel_err(y, ref) < 2e-5


def test_hyena_operator_vs_reference():
    from long_context_biomedical_imaging_amd import hyena
    g = Golden("hyena_op")
    torch.manual_seed(6)
    m = hyena.HyenaOperator(d_model=128, l_max=66000, filter_order=64, num_heads=2, num_blocks=1,
                            short_filter_order=5, bidrectional=True, dropout=0.0, filter_dropout=0.0, activation="id")
    m.load_state_dict(g.sd(), strict=False)   # z / t / deltas are deterministic buffers (checked on CPU)
    m = m.cuda()
    x = g.t("in/x").cuda().requires_grad_(True)
    out = m(x)
    assert rel_err(out, g.t("out/0")) < 1e-4
    out.backward(cotangents([out])[0].cuda())
    assert rel_err(x.grad, g.t("grad/in0")) < 2e-4
    for p in ("in_proj.weight", "filter_fn.bias", "short_filter.weight", "filter_fn.implicit_filter.0.weight"):
        assert rel_err(dict(m.named_parameters())[p].grad, g.t(f"grad/{p}")) < 5e-4, p
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out2 = m(g.t("in/x").cuda())
    assert rel_err(out2, g.t("out/0")) < 2e-2


def test_hyena_operator_autocast_grads_vs_reference(monkeypatch):
    """bf16 autocast (the training configuration) against the reference's fp32 golden gradients: the fused
    implicit filter (kernels.hyena_filter) is no further from them than the autocast module path of the same
    filter (LCI_FUSED_FILTER=0, the reference's own torch ops), output and every golden gradient."""
    from long_context_biomedical_imaging_amd import hyena
    g = Golden("hyena_op")
    torch.manual_seed(6)
    m = hyena.HyenaOperator(d_model=128, l_max=66000, filter_order=64, num_heads=2, num_blocks=1,
                            short_filter_order=5, bidrectional=True, dropout=0.0, filter_dropout=0.0, activation="id")
    m.load_state_dict(g.sd(), strict=False)
    m = m.cuda()
    names = ("in_proj.weight", "filter_fn.bias", "short_filter.weight", "filter_fn.implicit_filter.0.weight")
    errs = {}
    for fused in (False, True):
        monkeypatch.setenv("LCI_FUSED_FILTER", "1" if fused else "0")
        m.zero_grad(set_to_none=True)
        x = g.t("in/x").cuda().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            assert m.filter_fn.fused_filter_ok(x.shape[1]) == fused
            out = m(x)
        out.float().backward(cotangents([g.t("out/0")])[0].cuda())
        e = {"out": rel_err(out, g.t("out/0")), "in0": rel_err(x.grad, g.t("grad/in0"))}
        for p in names:
            e[p] = rel_err(dict(m.named_parameters())[p].grad, g.t(f"grad/{p}"))
        errs[fused] = e
    for k, e_mod in errs[False].items():
        assert errs[True][k] < 1.25 * e_mod + 2e-3, (k, errs[True][k], e_mod)


def test_hyena_lmax_error_matches_reference():
    from long_context_biomedical_imaging_amd import hyena
    m = hyena.HyenaOperator(d_model=64, l_max=128, num_heads=1, short_filter_order=5).cuda()
    with pytest.raises(AttributeError):
        m(torch.randn(1, 129, 64, device="cuda"))


def test_vit_hyena_encoder_vs_reference():
    from long_context_biomedical_imaging_amd import backbone_vit
    g = Golden("vit_enc_hyena")
    torch.manual_seed(4)
    m = backbone_vit.ViT_with_alt_ops(True, False, in_channels=1, img_size=(16, 16), patch_size=(2, 2),
                                      hidden_size=128, mlp_dim=256, num_layers=1, num_heads=2, dropout_rate=0.0,
                                      spatial_dims=2)
    m.load_state_dict(g.sd(), strict=False)
    m = m.cuda()
    outs = m(g.t("in/x").cuda())
    for i, (a, b) in enumerate(zip(outs, g.outs())):
        assert rel_err(a, b) < 1e-4, f"output {i}"


def test_vit_mamba_encoder_vs_reference():
    from long_context_biomedical_imaging_amd import backbone_vit
    g = Golden("vit_enc_mamba")
    m = backbone_vit.ViT_with_alt_ops(False, True, in_channels=1, img_size=(16, 16), patch_size=(2, 2),
                                      hidden_size=128, mlp_dim=256, num_layers=1, num_heads=2, dropout_rate=0.0,
                                      spatial_dims=2)
    m.load_state_dict(g.sd())
    m = m.cuda()
    outs = m(g.t("in/x").cuda())
    for i, (a, b) in enumerate(zip(outs, g.outs())):
        assert rel_err(a, b) < 1e-4, f"output {i}"


def test_compat_fftconv_ref_signature():
    """fftconv_ref(u, k, D, dropout_mask, gelu, k_rev) with the reference's 5-D (b, H, C, 1, L) call shape."""
    from long_context_biomedical_imaging_amd.compat import fftconv_ref
    g = Golden("fftconv_L1000")
    u = g.t("in/u").unsqueeze(3).cuda()
    y = fftconv_ref(u, g.t("in/k").cuda(), g.t("in/D").reshape(1, 64, 1).cuda(), dropout_mask=None, gelu=False)
    assert y.shape == u.shape
    assert rel_err(y[:, :, :, 0], g.t("out/y")) < 2e-5


def test_fftconv_c4_length_subset():
    """configs[3] length: L = 262144 (1024^2 patch 2), FFT n = 2^19 (n1 = 1024 column FFTs, in registers, n2 = 512 rows).
    Whole rows vs an fp64 torch.fft evaluation of the same causal convolution, plus 64 output positions of each
    row against the direct sum y[t] = sum_{s<=t} k[t-s] u[s] + D u[t]; gradients through the same path
    (adjoint rows vs fp64 FFT correlation). Tolerance rel-L2 2e-5 (as at L <= 65536)."""
    from long_context_biomedical_imaging_amd import kernels
    R, C, L = 2, 3, 262144
    torch.manual_seed(262144)
    u = torch.randn(R, C, L)
    k = torch.randn(C, L) * torch.exp(-torch.linspace(0, 12, L))[None]
    D = torch.randn(C)
    uc, kc, Dc = (t.cuda().requires_grad_(True) for t in (u, k, D))
    y = kernels.fftconv(uc, kc, Dc)
    n = 2 * L
    ud, kd = u.double(), k.double()
    ref = torch.fft.irfft(torch.fft.rfft(ud, n) * torch.fft.rfft(kd, n), n)[..., :L] + ud * D.double()[:, None]
    assert rel_err(y, ref) < 2e-5
    g = torch.Generator().manual_seed(1)
    ts = torch.randint(0, L, (64,), generator=g).tolist() + [0, 1, L - 1]
    yc = y.detach().cpu().double()
    for t in ts:
        direct = (kd[:, :t + 1].flip(-1)[None] * ud[..., :t + 1]).sum(-1) + ud[..., t] * D.double()
        assert torch.allclose(yc[..., t], direct, rtol=1e-4, atol=1e-4 * direct.abs().max().item())
    cot = torch.randn(R, C, L)
    y.backward(cot.cuda())
    cd = cot.double()
    # du = corr(cot, k) + D cot ; dk = sum_rows corr(cot, u) ; dD = sum cot u
    du = torch.fft.irfft(torch.fft.rfft(cd.flip(-1), n) * torch.fft.rfft(kd, n), n)[..., :L].flip(-1) + cd * D.double()[:, None]
    dk = torch.fft.irfft(torch.fft.rfft(cd.flip(-1), n) * torch.fft.rfft(ud, n), n)[..., :L].flip(-1).sum(0)
    dD = (cd * ud).sum((0, 2))
    assert rel_err(uc.grad, du) < 1e-4
    assert rel_err(kc.grad, dk) < 1e-4
    assert rel_err(Dc.grad, dD) < 1e-4


@pytest.mark.parametrize("BB,L,H,hd,K,dtype", [(2, 1000, 6, 64, 5, torch.float32), (1, 4099, 2, 32, 3, torch.float32),
                                              (2, 777, 6, 64, 5, torch.bfloat16), (1, 300, 1, 64, 8, torch.float32),
                                              (1, 129, 3, 64, 1, torch.float32)])
def test_hyena_short_conv_gate_vs_torch(BB, L, H, hd, K, dtype):
    """hyena_pre (register-ring kernels) vs a torch fp64 restatement of hyena.py:317-333 (causal depthwise conv1d,
    split x1 / x2 / v per head, v * x1): forward and the gradients of z, weight and bias. Ragged token tiles,
    head dims 32 / 64, filter orders 1-8."""
    from long_context_biomedical_imaging_amd import kernels
    torch.manual_seed(L + K)
    D = H * hd
    z = torch.randn(BB, L, 3 * D).to(dtype)
    w = torch.randn(3 * D, 1, K) * 0.5
    b = torch.randn(3 * D) * 0.1
    zc, wc, bc = (t.cuda().requires_grad_(True) for t in (z, w, b))
    vg, x2 = kernels.hyena_pre(zc, wc, bc, H)
    gv, g2 = torch.randn(BB, D, L), torch.randn(BB, L, D)
    (vg * gv.cuda()).sum().add_((x2.float() * g2.cuda()).sum()).backward()
    zr, wr, br = (t.double().requires_grad_(True) for t in (z.float(), w, b))
    conv = torch.nn.functional.conv1d(zr.transpose(1, 2), wr, br, padding=K - 1, groups=3 * D)[..., :L]
    conv = conv.view(BB, H, 3, hd, L)
    x1r, x2r, vr = conv[:, :, 0].reshape(BB, D, L), conv[:, :, 1].reshape(BB, D, L), conv[:, :, 2].reshape(BB, D, L)
    vgr = vr * x1r
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel_err(vg, vgr) < tol
    assert rel_err(x2.float(), x2r.transpose(1, 2)) < tol
    ((vgr * gv.double()).sum() + (x2r.transpose(1, 2) * g2.double()).sum()).backward()
    assert rel_err(zc.grad.float(), zr.grad) < max(tol, 1e-5)
    # bf16: autograd hands the kernel the x2 cotangent rounded to bf16 (x2 is bf16), so dw / db of the x2
    # channels carry that rounding (~2^-9 relative)
    tw = 1e-4 if dtype == torch.float32 else 1e-2
    assert rel_err(wc.grad, wr.grad) < tw
    assert rel_err(bc.grad, br.grad) < tw


@pytest.mark.parametrize("R,C,L", [(3072, 32, 512), (40, 32, 343), (7, 3, 64), (33, 32, 16), (5, 8, 49),
                                   (64, 64, 100), (2, 4, 1), (9, 5, 511)])
def test_direct_long_conv_vs_oracle(R, C, L):
    """The direct (Toeplitz, f32 MFMA) long conv taken for Swin-window rows (L <= 512; backbone_swin.py:361-362): y,
    du, dk and dD against fp64 autograd of the oracle's fftconv (hyena.py:32-51 semantics) at the f32 bounds of the
    FFT path (2e-5 outputs, 1e-4 gradients), plus the FFT path itself on the same rows (LCI_DIRECT_CONV=0)."""
    from long_context_biomedical_imaging_amd import kernels
    assert L <= kernels.direct_conv_max_len()
    torch.manual_seed(R + C + L)
    u = torch.randn(R, C, L)
    k = torch.randn(C, L) * torch.exp(-torch.linspace(0, 4, L))[None]
    D = torch.randn(C)
    uc, kc, Dc = (t.cuda().requires_grad_(True) for t in (u, k, D))
    y = kernels._DirectConv.apply(uc, kc, Dc)
    ur, kr, Dr = (t.double().requires_grad_(True) for t in (u, k, D))
    ref = oh.fftconv(ur[None], kr, Dr)[0] if R * C * L <= 2 ** 22 else None
    if ref is None:   # large case: direct fp64 sums on a row subset
        rows = torch.tensor([0, 1, R // 2, R - 1])
        ref_rows = oh.fftconv(u[rows].double()[None], k.double(), D.double())[0]
        assert rel_err(y[rows], ref_rows) < 2e-5
    else:
        assert rel_err(y, ref) < 2e-5
        cot = torch.randn(R, C, L)
        y.backward(cot.cuda())
        (ref * cot.double()).sum().backward()
        assert rel_err(uc.grad, ur.grad) < 1e-4
        assert rel_err(kc.grad, kr.grad) < 1e-4
        assert rel_err(Dc.grad, Dr.grad) < 1e-4
    yf = kernels._FFTConv.apply(u.cuda(), k.cuda(), D.cuda())
    assert rel_err(y, yf) < 2e-5
