"""HIP LayerNorm of TransformerBlock (backbone_vit.py:253-263) against torch's fp32 layer_norm.

f32 output: rel-L2 <= 1e-6 and max |err| <= 1e-5. bf16 output (the autocast operand of the next Linear): each
element is the bf16 rounding of the fp32 result, so it may differ from torch's rounding only where the two f32
values straddle a rounding boundary: |err| <= 1 bf16 ulp of the reference + 1e-5 (the f32 absolute error where
y = n gamma + beta cancels to near zero) everywhere, >= 99.5 % bit-equal.
Gradients (dx, dgamma, dbeta) vs torch autograd in fp64 on the same cotangent: rel-L2 <= 1e-5.
"""
import pytest
import torch
import torch.nn.functional as F

from golden_util import rel_err

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,C", [(1, 384), (4099, 384), (513, 192), (257, 768), (130, 1024), (77, 100),
                                    (2 * 65536, 384), (97, 1536), (33, 2048), (41, 1030), (19, 2052), (25, 6)])
@pytest.mark.parametrize("bf16", [False, True])
def test_layernorm_vs_torch(rows, C, bf16):
    from long_context_biomedical_imaging_amd import kernels
    torch.manual_seed(rows + C)
    x = (torch.randn(rows, C) * 3 + 0.5).cuda()
    w = (1 + 0.1 * torch.randn(C)).cuda()
    b = (0.1 * torch.randn(C)).cuda()
    xr, wr, br = [t.double().requires_grad_(True) for t in (x, w, b)]
    ref = F.layer_norm(xr, (C,), wr, br, 1e-5)
    xc, wc, bc = [t.clone().requires_grad_(True) for t in (x, w, b)]
    y = kernels.layer_norm(xc, wc, bc, 1e-5, bf16)
    if bf16:
        assert y.dtype == torch.bfloat16
        r32 = ref.detach().float()
        exact = (y == r32.to(torch.bfloat16)).float().mean().item()
        ulp = r32.abs().clamp_min(1e-30) * 2.0 ** -7
        assert ((y.float() - r32).abs() <= ulp + 1e-5).all()
        assert exact >= 0.995, exact
    else:
        assert y.dtype == torch.float32
        assert rel_err(y, ref) < 1e-6
        assert (y.double() - ref.detach()).abs().max().item() < 1e-5
    dy = torch.randn(rows, C).cuda().to(y.dtype)
    y.backward(dy)
    ref.backward(dy.double())
    assert rel_err(xc.grad, xr.grad) < 1e-5
    assert rel_err(wc.grad, wr.grad) < 1e-5
    assert rel_err(bc.grad, br.grad) < 1e-5


def test_token_layernorm_module_autocast():
    """TransformerBlock's norm under bf16 autocast hands the Linear the bf16 operand; outside autocast f32."""
    from long_context_biomedical_imaging_amd import backbone_vit
    torch.manual_seed(0)
    m = backbone_vit.TokenLayerNorm(384).cuda()
    ref = torch.nn.LayerNorm(384).cuda()
    ref.load_state_dict(m.state_dict())
    x = torch.randn(2, 1000, 384, device="cuda")
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
        lin = torch.nn.Linear(384, 8).cuda()
        r = ref(x)
        assert y.dtype == torch.bfloat16 and r.dtype == torch.float32
        assert torch.allclose(lin(y).float(), lin(r).float(), atol=0, rtol=0) or \
            rel_err(lin(y), lin(r)) < 1e-3
    y32 = m(x)
    assert y32.dtype == torch.float32 and rel_err(y32, ref(x)) < 1e-6


@pytest.mark.parametrize("bf16", [False, True])
def test_residual_layernorm_fused_gradient(bf16):
    """(h, y) = residual_layer_norm(x): h is x, and x.grad = dh + LN-backward(dy) computed in one kernel; checked
    on a block x + f(LN(x)) against fp64 torch autograd (rel-L2 <= 1e-5 on x / gamma / beta grads)."""
    from long_context_biomedical_imaging_amd import kernels
    torch.manual_seed(7)
    rows, C = 3001, 384
    x = (torch.randn(rows, C) * 2).cuda()
    w = (1 + 0.1 * torch.randn(C)).cuda()
    b = (0.1 * torch.randn(C)).cuda()
    P = (torch.randn(C, C) / C ** 0.5).cuda()
    cot = torch.randn(rows, C).cuda()
    xr, wr, br = [t.double().requires_grad_(True) for t in (x, w, b)]
    yr = F.layer_norm(xr, (C,), wr, br, 1e-5)
    (((xr + yr @ P.double()) * cot.double()).sum()).backward()
    xc, wc, bc = [t.clone().requires_grad_(True) for t in (x, w, b)]
    h, y = kernels.residual_layer_norm(xc, wc, bc, 1e-5, bf16)
    assert torch.equal(h, xc)
    (((h + y.float() @ P) * cot).sum()).backward()
    tol = 1e-5 if not bf16 else 1e-2   # bf16 y carries the operand rounding into the product's gradient path
    assert rel_err(xc.grad, xr.grad) < tol
    assert rel_err(wc.grad, wr.grad) < tol
    assert rel_err(bc.grad, br.grad) < tol


def test_residual_layernorm_unused_output_and_offset_cotangent():
    """LN output unused: the residual gradient passes through unchanged (no LN backward over zeros). A bf16
    cotangent that is a contiguous view at an odd storage offset is realigned before the kernel's vector loads."""
    from long_context_biomedical_imaging_amd import kernels
    torch.manual_seed(3)
    rows, C = 257, 384
    x = torch.randn(rows, C, device="cuda", requires_grad=True)
    w, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    h, _y = kernels.residual_layer_norm(x, w, b, 1e-5, True)
    g = torch.randn(rows, C, device="cuda")
    h.backward(g)
    assert torch.equal(x.grad, g)
    xr = x.detach().double().requires_grad_(True)
    ref = F.layer_norm(xr, (C,), w.double(), b.double(), 1e-5)
    big = torch.randn(rows * C + 1, device="cuda").to(torch.bfloat16)
    dy = big[1:].view(rows, C)          # contiguous, 2-byte offset
    assert dy.data_ptr() % 8 != 0
    x2 = x.detach().clone().requires_grad_(True)
    y2 = kernels.layer_norm(x2, w, b, 1e-5, True)
    y2.backward(dy)
    ref.backward(dy.double())
    assert rel_err(x2.grad, xr.grad) < 1e-5


def test_swin_large_stage4_block():
    """The Swin 'large' preset's last stage has C = 192 * 8 = 1536 channels (> the 1024 the first LayerNorm
    kernel handled): a SwinTransformerBlock of that width runs fwd + bwd on the HIP LayerNorm."""
    from long_context_biomedical_imaging_amd import backbone_swin
    torch.manual_seed(0)
    blk = backbone_swin.SwinTransformerBlock(False, False, 1536, 48, (7, 7, 7), (0, 0, 0)).cuda()
    x = torch.randn(1, 4, 4, 4, 1536, device="cuda", requires_grad=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = blk(x, None)
    y.float().square().mean().backward()
    assert y.shape == x.shape and torch.isfinite(x.grad).all()


@pytest.mark.parametrize("adtype", [torch.float32, torch.bfloat16])
def test_add_residual_layernorm(adtype):
    """(x, y) = add_residual_layer_norm(h, a): x = h + a computed in the LN forward kernel (bitwise torch's f32
    add), y = LN(x) as layer_norm; gradients of h, a, gamma, beta on a block (h + a) + f(LN(h + a)) against fp64
    torch autograd (rel-L2 <= 1e-5), a's gradient in a's dtype."""
    from long_context_biomedical_imaging_amd import kernels
    torch.manual_seed(11)
    rows, C = 2051, 384
    h = (torch.randn(rows, C) * 2).cuda()
    a = torch.randn(rows, C).cuda().to(adtype)
    w = (1 + 0.1 * torch.randn(C)).cuda()
    b = (0.1 * torch.randn(C)).cuda()
    P = (torch.randn(C, C) / C ** 0.5).cuda()
    cot = torch.randn(rows, C).cuda()
    hr, ar, wr, br = [t.double().requires_grad_(True) for t in (h, a.float(), w, b)]
    xr = hr + ar
    yr = F.layer_norm(xr, (C,), wr, br, 1e-5)
    (((xr + yr @ P.double()) * cot.double()).sum()).backward()
    hc, ac, wc, bc = [t.clone().requires_grad_(True) for t in (h, a, w, b)]
    x, y = kernels.add_residual_layer_norm(hc, ac, wc, bc, 1e-5, False)
    assert torch.equal(x, h + a)
    assert rel_err(y, F.layer_norm(h + a, (C,), w, b, 1e-5)) < 1e-6
    (((x + y @ P) * cot).sum()).backward()
    assert ac.grad.dtype == adtype
    # the bf16 branch gradient is written by the LN backward kernel: h's f32 gradient rounded once
    assert torch.equal(ac.grad, hc.grad.to(adtype))
    assert rel_err(hc.grad, hr.grad) < 1e-5
    assert rel_err(ac.grad, ar.grad) < (1e-5 if adtype == torch.float32 else 1e-2)
    assert rel_err(wc.grad, wr.grad) < 1e-5
    assert rel_err(bc.grad, br.grad) < 1e-5


@pytest.mark.parametrize("add", [False, True])
def test_residual_layernorm_tap_alias(add):
    """tap=True returns a second alias of the LN input (a recorded hidden state read outside the block): its gradient
    is summed inside the LN backward kernel (lci_layernorm_bwd dres2), bitwise the autograd sum of the two consumers'
    gradients that the one-alias form gets."""
    from long_context_biomedical_imaging_amd import kernels
    torch.manual_seed(21)
    rows, C = 3001, 384
    h0 = (torch.randn(rows, C) * 2).cuda()
    a0 = torch.randn(rows, C).cuda().to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(C)).cuda()
    b = (0.1 * torch.randn(C)).cuda()
    P = (torch.randn(C, C) / C ** 0.5).cuda()
    c1, c2 = torch.randn(rows, C).cuda(), torch.randn(rows, C).cuda()
    grads = []
    for tap in (False, True):
        h = h0.clone().requires_grad_(True)
        a = a0.clone().requires_grad_(True)
        if add:
            out = kernels.add_residual_layer_norm(h, a, w, b, 1e-5, False, tap)
        else:
            out = kernels.residual_layer_norm(h, w, b, 1e-5, False, tap)
        x, t, y = out if tap else (out[0], out[0], out[1])
        ((x * c1).sum() + (t * t * c2).sum() + (y @ P).square().sum()).backward()
        grads.append((h.grad.clone(), a.grad.clone() if add else None))
    assert torch.equal(grads[0][0], grads[1][0])
    if add:
        assert torch.equal(grads[0][1], grads[1][1])
