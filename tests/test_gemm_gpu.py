"""Projection GEMM (csrc/gemm.hip, lci_gemm_bt): y = x . w^T + b in bf16 with f32 accumulation, the forward and data
gradient of every token-wise nn.Linear under autocast whose output width is a multiple of 384 (SABlock qkv / out_proj
backbone_vit.py:166-167, MLPBlock :249, Hyena in/out_proj hyena.py:278-279, Mamba in/out_proj mamba.py:60-64,90).

Against an fp64 product of the same bf16 operands: every element within one bf16 rounding of the exact value plus an
f32-accumulation allowance (|err| <= 2^-8 |ref| + 2^-16 sum|x||w|), ragged M (tile tails, M < one tile), strided x
rows (a column slice), every feature tile of N = 384 .. 1536 and K = 96 .. 1536. The TokenLinear module under autocast
(forward + input / weight / bias gradients) against torch's own autocast nn.Linear on the GPU.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _check(y, x, w, b):
    ref = x.double() @ w.double().t()
    if b is not None:
        ref = ref + b.double()
    bound = ref.abs() * 2.0 ** -8 + (x.double().abs() @ w.double().abs().t()) * 2.0 ** -16 + 1e-30
    err = (y.double() - ref).abs()
    bad = (err > bound).sum().item()
    assert bad == 0, f"{bad} elements outside the bound; max err {err.max().item():.3e}"


@pytest.mark.parametrize("M,N,K,bias,pad", [(1, 384, 384, True, 0), (255, 384, 384, False, 0), (256, 1152, 384, True, 0),
                                            (1000, 1536, 384, True, 64), (4173, 384, 1536, False, 0),
                                            (777, 768, 96, True, 8), (3001, 384, 320, True, 0),
                                            (2500, 384, 1152, True, 0), (131072, 1152, 384, True, 0),
                                            # 256-feature tiles (N % 384 != 0: ConvTranspose-as-GEMM widths 8 Cout)
                                            (3001, 512, 384, True, 0), (700, 1024, 256, False, 8),
                                            (20000, 2048, 384, True, 0), (513, 4096, 512, True, 0)])
def test_gemm_bt_vs_fp64(M, N, K, bias, pad):
    from long_context_biomedical_imaging_amd import kernels
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    xf = torch.randn(M, K + pad, device="cuda", generator=g).to(torch.bfloat16)
    x = xf[:, :K]                                  # strided rows when pad > 0
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16) if bias else None
    assert kernels.gemm_bt_supported(x, N, K)
    y = kernels.gemm_bt(x, w, b)
    if M > 20000:   # check a row subset at the large size (tiles spread over every XCD and workgroup)
        rows = torch.cat([torch.arange(0, 512), torch.arange(M // 2 - 300, M // 2 + 300), torch.arange(M - 700, M)]).cuda()
        _check(y[rows], x[rows], w, b)
    else:
        _check(y, x, w, b)


@pytest.mark.parametrize("D,H,M", [(384, 1152, 3000), (1536, 384, 2048), (384, 384, 513)])
def test_token_linear_autocast_fwd_bwd(D, H, M, monkeypatch):
    """TokenLinear (kernels.linear) on lci_gemm_bt under bf16 autocast vs torch's autocast nn.Linear, same weights."""
    from long_context_biomedical_imaging_amd import blocks, kernels
    monkeypatch.setattr(kernels, "HIP_GEMM", True)
    monkeypatch.setattr(kernels, "GEMM_BT_MIN_TILES", 0)   # these token counts are below the routing threshold
    torch.manual_seed(D + H)
    lin = blocks.TokenLinear(D, H).cuda()
    ref = torch.nn.Linear(D, H).cuda()
    ref.load_state_dict(lin.state_dict())
    x = torch.randn(2, M, D, device="cuda")
    x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y1 = lin(x1)
        y2 = ref(x2)
    assert kernels.gemm_bt_supported(x1.to(torch.bfloat16).reshape(-1, D), H, D)
    assert y1.dtype == y2.dtype == torch.bfloat16
    e = ((y1.float() - y2.float()).norm() / y2.float().norm()).item()
    assert e < 4e-3, f"forward rel {e:.3e}"
    gy = torch.randn_like(y1)
    y1.backward(gy)
    y2.backward(gy)
    for a, b, nm in ((x1.grad, x2.grad, "dx"), (lin.weight.grad, ref.weight.grad, "dW"), (lin.bias.grad, ref.bias.grad, "db")):
        e = ((a.float() - b.float()).norm() / b.float().norm()).item()
        assert e < 1e-2, f"{nm} rel {e:.3e}"


def test_gemm_bt_deterministic():
    from long_context_biomedical_imaging_amd import kernels
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(5000, 384, device="cuda", generator=g).to(torch.bfloat16)
    w = torch.randn(1536, 384, device="cuda", generator=g).to(torch.bfloat16)
    assert torch.equal(kernels.gemm_bt(x, w), kernels.gemm_bt(x, w))


def test_gemm_bt_supported_shapes():
    from long_context_biomedical_imaging_amd import _lib
    lib = _lib.load()
    assert lib.lci_gemm_bt_supported(384, 192) and not lib.lci_gemm_bt_supported(4224, 1536)
    assert not lib.lci_gemm_bt_supported(384, 48) and not lib.lci_gemm_bt_supported(400, 384)
    assert lib.lci_gemm_bt_supported(2048, 384) and lib.lci_gemm_bt_supported(512, 64)
    assert not lib.lci_gemm_bt_supported(640, 384) and not lib.lci_gemm_bt_supported(4352, 384)


@pytest.mark.parametrize("M,N,K", [(70001, 256, 32), (66000, 512, 256), (131072, 384, 384)])
def test_gemm_bt_acc_is_the_autograd_sum(M, N, K):
    """lci_gemm_bt_acc: y <- bf16(y + bf16(x . w^T)), bitwise the sum autograd forms of y and lci_gemm_bt's product
    (UnetResBlock's 1x1 residual data gradient added into conv1's)."""
    from long_context_biomedical_imaging_amd import _lib, kernels
    g = torch.Generator(device="cuda").manual_seed(M + N)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    y0 = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    ref = (y0.float() + kernels.gemm_bt(x, w).float()).to(torch.bfloat16)
    y = y0.clone()
    _lib.call("lci_gemm_bt_acc", x.data_ptr(), K, w.data_ptr(), y.data_ptr(), N, M, N, K, _lib.stream_of(x))
    assert torch.equal(y, ref)
