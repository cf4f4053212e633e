"""Token-wise Linear on the HIP weight-gradient kernel (lci_linear_wgrad; blocks.TokenLinear).

- dW = dY^T X and db = sum dY vs an fp64 product of the same bf16 operands, for every tile the kernel picks: the
  ViT / Mamba / Hyena / Swin projection shapes, ragged token counts (not multiples of the 64-row slab or of the
  split), N / K not multiples of the tile (x_proj 40 x 192, dt_proj 192 x 24) and a strided operand view (dt_proj
  reads x_proj's output columns [0, 24) of a 40-wide row). Bound: |err| <= 1e-5 * (|dY|^T |X|) + 1e-6 elementwise
  (f32 accumulation of exact bf16 products).
- At the C5 token count (M = 2^21, 384 x 384) the same bound.
- TokenLinear under bf16 autocast vs nn.Linear under autocast (the reference path, backbone_vit.py:166-167):
  identical output and input gradient (the same hipBLASLt GEMMs), weight / bias gradients within the bf16 rounding
  the autocast GEMM applies to its dW (ours stay f32).
"""
import pytest
import torch

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
                                   (2049, 192, 768), (65, 768, 384), (1, 384, 384)])
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
def test_token_linear_matches_autocast_linear(N, K, bias):
    from long_context_biomedical_imaging_amd.blocks import TokenLinear
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
