"""Small / narrow projection GEMM (csrc/gemm.hip, lci_gemm_bt_small, round 6): y = x . w^T + b in bf16 with f32
accumulation for the shapes lci_gemm_bt's persistent 256 x 384 tiles do not take or fill -- the Swin stage-3 / 4
projections and data gradients (backbone_swin.py:339-359 qkv / proj and the Mlp, 4096 / 512 tokens at C3) and the
decoder heads' 96 / 192 / 288-wide 1x1 convolutions (MONAI UnetResBlock conv3 / UnetOutBlock, enhance_heads.py:30-356).

Against an fp64 product of the same bf16 operands with test_gemm_gpu's bound (one bf16 rounding plus an f32
accumulation allowance), ragged M (partial 32-token blocks, M = 1), strided x rows, every NBW tile (N / 32 divisible by
4, 3, 2 or only 1); the accumulate form bitwise against the sum autograd forms; TokenLinear at the Swin stage-3 size
under autocast against torch's nn.Linear; and the routing (which kernel a shape takes).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _check(y, x, w, b):   # (test_gemm_gpu's bound)
    ref = x.double() @ w.double().t()
    if b is not None:
        ref = ref + b.double()
    bound = ref.abs() * 2.0 ** -8 + (x.double().abs() @ w.double().abs().t()) * 2.0 ** -16 + 1e-30
    err = (y.double() - ref).abs()
    bad = (err > bound).sum().item()
    assert bad == 0, f"{bad} elements outside the bound; max err {err.max().item():.3e}"


@pytest.mark.parametrize("M,N,K,bias,pad", [
    (1, 32, 16, True, 0), (37, 96, 96, False, 0), (4096, 384, 384, True, 0), (4096, 1536, 384, True, 0),
    (4096, 384, 1536, False, 0), (4096, 1152, 384, True, 8), (512, 768, 768, True, 0), (512, 3072, 768, True, 0),
    (512, 768, 3072, False, 0), (4099, 288, 96, True, 0), (70000, 96, 192, False, 0), (65537, 192, 96, True, 16),
    (3000, 160, 48, True, 0), (1000, 64, 32, False, 0), (262144, 96, 384, False, 0)])
def test_gemm_small_vs_fp64(M, N, K, bias, pad):
    from long_context_biomedical_imaging_amd import kernels
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    xf = torch.randn(M, K + pad, device="cuda", generator=g).to(torch.bfloat16)
    x = xf[:, :K]
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16) if bias else None
    assert kernels.gemm_small_supported(x, N, K)
    y = kernels.gemm_small(x, w, b)
    if M > 20000:
        rows = torch.cat([torch.arange(0, 700), torch.arange(M // 2 - 300, M // 2 + 300), torch.arange(M - 700, M)]).cuda()
        _check(y[rows], x[rows], w, b)
    else:
        _check(y, x, w, b)


@pytest.mark.parametrize("M,N,K", [(4096, 96, 192), (70001, 192, 96), (33, 288, 96)])
def test_gemm_small_acc_is_the_autograd_sum(M, N, K):
    """lci_gemm_bt_small_acc: y <- bf16(y + bf16(x . w^T)), bitwise the sum of y and lci_gemm_bt_small's product."""
    from long_context_biomedical_imaging_amd import kernels
    g = torch.Generator(device="cuda").manual_seed(M + N)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    y0 = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    ref = (y0.float() + kernels.gemm_small(x, w).float()).to(torch.bfloat16)
    y = y0.clone()
    assert kernels.gemm_small(x, w, out=y) is y
    assert torch.equal(y, ref)


def test_gemm_small_deterministic_and_supported():
    from long_context_biomedical_imaging_amd import _lib, kernels
    lib = _lib.load()
    assert lib.lci_gemm_bt_small_supported(96, 16) and lib.lci_gemm_bt_small_supported(32, 3072)
    assert not lib.lci_gemm_bt_small_supported(48, 96) and not lib.lci_gemm_bt_small_supported(96, 8)
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(5000, 384, device="cuda", generator=g).to(torch.bfloat16)
    w = torch.randn(96, 384, device="cuda", generator=g).to(torch.bfloat16)
    assert torch.equal(kernels.gemm_small(x, w), kernels.gemm_small(x, w))


@pytest.mark.parametrize("D,H,M", [(384, 1152, 4096), (1536, 384, 4096), (768, 3072, 512), (96, 192, 9000)])
def test_token_linear_small_autocast_fwd_bwd(D, H, M, monkeypatch):
    """TokenLinear (kernels.linear) at the Swin stage-3 / 4 and decoder sizes -- routed to lci_gemm_bt_small (opt-in,
    LCI_SMALL_GEMM=1), forward and data gradient -- under bf16 autocast against torch's autocast nn.Linear with the
    same weights."""
    from long_context_biomedical_imaging_amd import blocks, kernels
    monkeypatch.setattr(kernels, "SMALL_GEMM", True)
    torch.manual_seed(D + H)
    lin = blocks.TokenLinear(D, H).cuda()
    ref = torch.nn.Linear(D, H).cuda()
    ref.load_state_dict(lin.state_dict())
    x = torch.randn(1, M, D, device="cuda")
    x2d = x.reshape(-1, D).to(torch.bfloat16)
    assert not (kernels.gemm_bt_preferred(M, H) and kernels.gemm_bt_supported(x2d, H, D))
    dy2d = torch.empty(M, H, device="cuda", dtype=torch.bfloat16)
    assert kernels.gemm_small_supported(x2d, H, D) and kernels.gemm_small_supported(dy2d, D, H)
    x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    kernels.KernelTimer.reset()
    kernels.KernelTimer.enabled = True
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y1 = lin(x1)
            y2 = ref(x2)
        gy = torch.randn_like(y1)
        y1.backward(gy)
        y2.backward(gy)
        torch.cuda.synchronize()
        calls = kernels.KernelTimer.summary().get("gemm_bt_small", {}).get("calls", 0)
    finally:
        kernels.KernelTimer.enabled = False
    assert calls == 2, f"forward + data gradient on lci_gemm_bt_small: {calls} calls"
    e = ((y1.float() - y2.float()).norm() / y2.float().norm()).item()
    assert e < 4e-3, f"forward rel {e:.3e}"
    for a, b, nm in ((x1.grad, x2.grad, "dx"), (lin.weight.grad, ref.weight.grad, "dW"), (lin.bias.grad, ref.bias.grad, "db")):
        e = ((a.float() - b.float()).norm() / b.float().norm()).item()
        assert e < 1e-2, f"{nm} rel {e:.3e}"
