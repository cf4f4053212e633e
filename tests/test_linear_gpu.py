"""Token-wise Linear on the HIP weight-gradient kernel (lci_linear_wgrad; blocks.TokenLinear).

- dW = dY^T X and db = sum dY vs an fp64 product of the same bf16 operands, for every tile the kernel picks: the
  ViT / Mamba / Hyena / Swin projection shapes, ragged token counts (not multiples of the 64-row slab or of the
  split), N / K not multiples of the tile (x_proj 40 x 192, dt_proj 192 x 24) and a strided operand view (dt_proj
  reads x_proj's output columns [0, 24) of a 40-wide row). Bound: |err| <= 1e-5 * (|dY|^T |X|) + 1e-6 elementwise
  (f32 accumulation of exact bf16 products).
- At the C5 token count (M = 2^21, 384 x 384) the same bound.
- TokenLinear under bf16 autocast vs nn.Linear under autocast (the reference path, backbone_vit.py:166-167), with
  the forward / data-gradient GEMMs on hipBLASLt (LCI_HIP_GEMM=0; lci_gemm_bt's own parity is tests/test_gemm_gpu.py):
  identical output and input gradient, weight / bias gradients within the bf16 rounding the autocast GEMM applies to
  its dW (ours stay f32).
"""
import pytest
import torch

from golden_util import rel_err

pytestmark = pytest.mark.gpu


def _check(dy, x, bias):
    from long_context_biomedical_imaging_amd import kernels
    assert kernels.linear_wgrad_supported(dy, x)
    dw, db = kernels.linear_wgrad(dy, x, bias)
    ref = dy.double().t() @ x.double()
    bound = dy.double().abs().t() @ x.double().abs()
    err = (dw.double() - ref).abs()
    assert (err <= 1e-5 * bound + 1e-6).all(), f"dW max err {err.max().item():.3e}"
    if bias:
        rb = dy.double().sum(0)
        eb = (db.double() - rb).abs()
        assert (eb <= 1e-5 * dy.double().abs().sum(0) + 1e-6).all(), f"db max err {eb.max().item():.3e}"


@pytest.mark.parametrize("M,N,K", [(1000, 384, 384), (4099, 1536, 384), (3001, 384, 1536), (2500, 1152, 384),
                                   (777, 40, 192), (70001, 384, 384), (300, 288, 96), (1234, 96, 96),
                                   (2049, 192, 768), (65, 768, 384), (1, 384, 384),
                                   # narrow outputs (any padding): Swin-recipe Mamba x_proj / dt_proj gradients
                                   (5003, 24, 48), (4000, 48, 8), (3333, 32, 96), (2999, 96, 16), (1 << 19, 24, 48)])
def test_linear_wgrad_vs_fp64(M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    dy = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    _check(dy, x, bias=True)
    _check(dy, x, bias=False)


def test_linear_wgrad_strided_dt_proj_view():
    g = torch.Generator(device="cuda").manual_seed(7)
    M = 5000
    xdbl = torch.randn(M, 40, device="cuda", generator=g).to(torch.bfloat16)
    dy = torch.randn(M, 192, device="cuda", generator=g).to(torch.bfloat16)
    _check(dy, xdbl[:, :24], bias=True)


def test_linear_wgrad_c5_tokens():
    g = torch.Generator(device="cuda").manual_seed(21)
    M = 1 << 21
    dy = torch.randn(M, 384, device="cuda", generator=g).to(torch.bfloat16)
    x = torch.randn(M, 384, device="cuda", generator=g).to(torch.bfloat16)
    _check(dy, x, bias=True)


@pytest.mark.parametrize("N,K,bias", [(1152, 384, False), (384, 384, True), (1536, 384, True), (40, 192, False)])
def test_token_linear_matches_autocast_linear(N, K, bias, monkeypatch):
    from long_context_biomedical_imaging_amd import kernels
    from long_context_biomedical_imaging_amd.blocks import TokenLinear
    monkeypatch.setattr(kernels, "HIP_GEMM", False)   # hipBLASLt forward / dX: bitwise torch's (lci_gemm_bt: test_gemm_gpu)
    torch.manual_seed(0)
    ref = torch.nn.Linear(K, N, bias=bias).cuda()
    mine = TokenLinear(K, N, bias=bias).cuda()
    mine.load_state_dict(ref.state_dict())
    x = torch.randn(2, 3000, K, device="cuda")
    gy = torch.randn(2, 3000, N, device="cuda").to(torch.bfloat16)
    outs = []
    for m in (ref, mine):
        xi = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(xi)
        y.backward(gy)
        outs.append((y.detach(), xi.grad, m.weight.grad, m.bias.grad if bias else None))
    (y0, dx0, dw0, db0), (y1, dx1, dw1, db1) = outs
    assert y1.dtype == y0.dtype == torch.bfloat16 and torch.equal(y0, y1)
    assert torch.equal(dx0, dx1)
    assert dw1.dtype == torch.float32
    # dw0 is the bf16 rounding of an f32 sum in another order: half an ulp plus the f32 reassociation bound
    g2, x2 = gy.reshape(-1, N).float().abs(), x.reshape(-1, K).to(torch.bfloat16).float().abs()
    assert ((dw1 - dw0).abs() <= 2 ** -8 * dw0.abs() + 1e-5 * (g2.t() @ x2)).all()
    if bias:
        assert ((db1 - db0).abs() <= 2 ** -8 * db0.abs() + 1e-5 * g2.sum(0)).all()


def _ulp_close(a, b, ulps=1):
    """|a - b| <= ulps bf16 ulps of max(|a|, |b|) (elementwise), plus a tiny absolute floor."""
    a, b = a.double(), b.double()
    tol = ulps * 2.0 ** -7 * torch.maximum(a.abs(), b.abs()) + 1e-30
    return ((a - b).abs() <= tol)


@pytest.mark.parametrize("M,N,K", [(2 * 64 ** 3, 2, 48), (524288, 2, 16), (1000, 1, 24), (777, 4, 256), (99, 3, 64)])
def test_pointwise_small_vs_autocast_linear(M, N, K):
    """The UNETR heads' 1x1 conv to N <= 4 channels (decoders._pointwise) vs F.linear under bf16 autocast."""
    from long_context_biomedical_imaging_amd import kernels
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda", generator=g) * K ** -0.5
    b = torch.randn(N, device="cuda", generator=g)
    gy = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    outs = []
    for hip in (True, False):
        xi, wi, bi = x.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = kernels.pointwise_small(xi, wi, bi) if hip else torch.nn.functional.linear(xi, wi, bi)
        y.backward(gy)
        outs.append((y.detach(), xi.grad, wi.grad, bi.grad))
    for name, a, r in zip(("y", "dx", "dW", "db"), outs[0], outs[1]):
        assert a.dtype == r.dtype and a.shape == r.shape, name
        e = ((a.double() - r.double()).norm() / r.double().norm()).item()
        assert e < 5e-3, f"{name}: rel-L2 {e:.3e}"   # bf16 outputs / dW, db rounded to bf16 by the reference


@pytest.mark.parametrize("Cin,Cout", [(1, 96), (192, 96), (3, 32), (2, 48), (6, 32)])
def test_decoder_pointwise_conv_grads(Cin, Cout):
    """decoders.Conv1x1 (UnetResBlock's 1x1 residual conv) on kernels.linear: forward and input gradient equal to
    the same 1x1 conv as F.linear under autocast (torch's GEMMs), weight / bias gradients within its bf16 rounding
    (Cin <= 4: the swapped-role lci_linear_small_bwd weight gradient; Cin = 6: zero-padded to 8 columns)."""
    from long_context_biomedical_imaging_amd import decoders
    torch.manual_seed(Cin)
    conv = decoders.Conv1x1(Cin, Cout, 1, 1, bias=True).cuda()
    x = torch.randn(1, Cin, 24, 20, 16, device="cuda").to(memory_format=torch.channels_last_3d)
    outs = []
    for hip in (True, False):
        conv.zero_grad()
        xi = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = conv(xi) if hip else torch.nn.functional.linear(
                xi.movedim(1, -1), conv.weight.reshape(Cout, Cin), conv.bias).movedim(-1, 1)
        gy = torch.randn(y.shape, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5)).to(y.dtype)
        y.backward(gy)
        outs.append((y.detach().float(), xi.grad.float(), conv.weight.grad.clone(), conv.bias.grad.clone()))
    for name, a, r in zip(("y", "dx", "dW", "db"), outs[0], outs[1]):
        e = ((a.double() - r.double()).norm() / r.double().norm()).item()
        assert e < 1e-2, f"{name}: rel-L2 {e:.3e}"


@pytest.mark.parametrize("nd,Cin,Cout,k", [(3, 96, 64, (2, 2, 2)), (3, 384, 128, (2, 2, 2)), (2, 64, 32, (2, 2))])
def test_conv_up_gemm_grads(nd, Cin, Cout, k):
    """decoders.ConvUp (kernel == stride transposed conv as one GEMM on kernels.linear, tap-major columns, bias in
    the GEMM) under bf16 autocast vs the fp32 transposed convolution on the same (bf16-representable) data."""
    from long_context_biomedical_imaging_amd import decoders
    torch.manual_seed(Cin + Cout)
    ct = (torch.nn.ConvTranspose3d if nd == 3 else torch.nn.ConvTranspose2d)(Cin, Cout, k, k, bias=True).cuda()
    with torch.no_grad():
        ct.weight.copy_(ct.weight.to(torch.bfloat16).float())
        ct.bias.copy_(ct.bias.to(torch.bfloat16).float())
    shape = (1, Cin, 10, 12, 6) if nd == 3 else (2, Cin, 20, 14)
    mf = torch.channels_last_3d if nd == 3 else torch.channels_last
    x = torch.randn(shape, device="cuda").to(torch.bfloat16).float().to(memory_format=mf)
    gshape = (shape[0], Cout) + tuple(s * kk for s, kk in zip(shape[2:], k))
    gy = torch.randn(gshape, device="cuda").to(torch.bfloat16)
    res = []
    for hip in (True, False):
        ct.zero_grad()
        xi = x.clone().requires_grad_(True)
        if hip:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = decoders._up_gemm(xi, ct.weight, ct.bias, k)
            y.backward(gy)
        else:   # fp32 reference: the same math as torch's transposed conv (tests/test_conv_cpu.py pins it to it)
            w2 = ct.weight.reshape(Cin, -1)
            yy = (xi.movedim(1, -1).reshape(-1, Cin) @ w2).view(shape[0], *shape[2:], Cout, *k)
            yy = yy.permute(0, 1, 5, 2, 6, 3, 7, 4) if nd == 3 else yy.permute(0, 1, 4, 2, 5, 3)
            y = (yy.reshape(shape[0], *gshape[2:], Cout) + ct.bias).movedim(-1, 1)
            y.backward(gy.float())
        res.append((y.detach().float(), xi.grad.float(), ct.weight.grad.clone(), ct.bias.grad.clone()))
    for name, a, r in zip(("y", "dx", "dW", "db"), res[0], res[1]):
        e = ((a.double() - r.double()).norm() / r.double().norm()).item()
        assert e < 1e-2, f"{name}: rel-L2 {e:.3e}"


def test_gelu_kernel_matches_torch_bf16():
    """lci_gelu_fwd / _bwd vs torch's bf16 GELU (approximate='none') and its autograd: torch's f32 opmath
    expression with the same erff / expf, so the bf16 results agree bitwise (one bf16 ulp allowed where the f32
    contraction order could round differently)."""
    from long_context_biomedical_imaging_amd import kernels
    torch.manual_seed(0)
    x = torch.randn(3, 1000, 1536, device="cuda") * 3
    x.view(-1)[:8] = torch.tensor([0.0, -0.0, 1e-30, -1e-30, 20.0, -20.0, 6.5, -6.5])
    x = x.to(torch.bfloat16)
    assert kernels.gelu_supported(x)
    xr = x.clone().requires_grad_(True)
    ref = torch.nn.functional.gelu(xr)
    xc = x.clone().requires_grad_(True)
    y = kernels.gelu(xc)
    ulp = ref.detach().float().abs() * 2.0 ** -7 + 1e-30
    assert bool(((y.float() - ref.detach().float()).abs() <= ulp).all())
    assert (y == ref).float().mean().item() > 0.999
    g = torch.randn_like(ref)
    ref.backward(g)
    y.backward(g)
    ulp = xr.grad.float().abs() * 2.0 ** -7 + 1e-30
    assert bool(((xc.grad.float() - xr.grad.float()).abs() <= ulp).all())
    assert (xc.grad == xr.grad).float().mean().item() > 0.999


def test_gelu_kernel_exhaustive_bf16():
    """Every finite bf16 input (|x| < 1e4): the HIP GELU (forward, and backward with a unit cotangent) within one bf16
    ulp of torch's and bitwise equal for > 99.5 % of the inputs."""
    from long_context_biomedical_imaging_amd import kernels
    bits = torch.arange(0, 65536, dtype=torch.int32).to(torch.int16)
    x = bits.view(torch.bfloat16).cuda()
    x = x[torch.isfinite(x.float()) & (x.float().abs() < 1e4)].contiguous()
    x = x[: x.numel() // 8 * 8].contiguous()
    ref = torch.nn.functional.gelu(x)
    y = kernels.gelu(x)
    d = (y.float() - ref.float()).abs()
    assert bool((d <= ref.float().abs() * 2.0 ** -7 + 1e-37).all())
    assert (y != ref).float().mean().item() < 5e-3
    xr = x.clone().requires_grad_(True)
    torch.nn.functional.gelu(xr).backward(torch.ones_like(x))
    xc = x.clone().requires_grad_(True)
    kernels.gelu(xc).backward(torch.ones_like(x))
    d = (xc.grad.float() - xr.grad.float()).abs()
    assert bool((d <= xr.grad.float().abs() * 2.0 ** -7 + 1e-37).all())
    assert (xc.grad != xr.grad).float().mean().item() < 5e-3


@pytest.mark.parametrize("nd,Cin,Cout,Cs,k", [(3, 64, 32, 32, (2, 2, 2)), (2, 48, 16, 24, (2, 2)), (3, 16, 8, 0, (2, 2, 2))])
def test_conv_up_interleave_and_cat_bit_exact(nd, Cin, Cout, Cs, k, monkeypatch):
    """lci_convup_interleave (the up-sampling GEMM's rows moved to the channels-last grid, optionally straight into
    UnetrUpBlock's torch.cat buffer) against the torch view/permute/reshape (+ cat) it replaces: pure data movement,
    so outputs and gradients (x, W, b, skip) are bitwise equal."""
    from long_context_biomedical_imaging_amd import decoders, kernels
    torch.manual_seed(Cin)
    ct = (torch.nn.ConvTranspose3d if nd == 3 else torch.nn.ConvTranspose2d)(Cin, Cout, k, k, bias=True).cuda()
    shape = (2, Cin, 5, 6, 3) if nd == 3 else (2, Cin, 9, 7)
    mf = torch.channels_last_3d if nd == 3 else torch.channels_last
    x = torch.randn(shape, device="cuda").to(torch.bfloat16).to(memory_format=mf)
    so = tuple(s * kk for s, kk in zip(shape[2:], k))
    skip = torch.randn(shape[0], Cs, *so, device="cuda").to(torch.bfloat16).to(memory_format=mf) if Cs else None
    gy = torch.randn(shape[0], Cout + Cs, *so, device="cuda").to(torch.bfloat16)
    res = []
    for hip in (True, False):
        if not hip:
            monkeypatch.setattr(kernels, "convup_interleave_supported", lambda *a: False)
        ct.zero_grad()
        xi = x.clone().requires_grad_(True)
        si = skip.clone().requires_grad_(True) if Cs else None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = decoders._up_gemm(xi, ct.weight, ct.bias, k, si)
        y.backward(gy)
        res.append((y.detach(), xi.grad, ct.weight.grad.clone(), ct.bias.grad.clone(), si.grad if Cs else None))
    for name, a, b in zip(("y", "dx", "dW", "db", "dskip"), res[0], res[1]):
        assert (a is None and b is None) or torch.equal(a, b), name


@pytest.mark.parametrize("bias", [True, False])
def test_linear_one_input_channel_outer_product(bias):
    """K = 1 (the 1-channel image into encoder1's 1x1 residual conv) runs as an outer product: bitwise the autocast
    F.linear result (the bf16 x bf16 product is exact in f32, both round the same f32 value once), weight / bias
    gradients within the bf16 rounding the autocast GEMM applies to its dW."""
    from long_context_biomedical_imaging_amd import kernels
    torch.manual_seed(4)
    x = torch.randn(70001, 1, device="cuda")
    w = torch.randn(96, 1, device="cuda", requires_grad=True)
    b = torch.randn(96, device="cuda", requires_grad=True) if bias else None
    w2 = w.detach().clone().requires_grad_(True)
    b2 = b.detach().clone().requires_grad_(True) if bias else None
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ref = torch.nn.functional.linear(x, w, b)
        y = kernels.linear(x, w2, b2)
    assert y.dtype == ref.dtype == torch.bfloat16
    assert torch.equal(y, ref)
    g = torch.randn_like(ref)
    ref.float().backward(g.float())
    y.float().backward(g.float())
    assert rel_err(w2.grad, w.grad) < 1e-2
    if bias:
        assert rel_err(b2.grad, b.grad) < 1e-2
