"""GPU parity of the decoder-head 3x3(x3) convolution (csrc/conv.hip) against torch's fp32 convolution on the
same bf16-rounded operands (MONAI-1.3 get_conv_layer(kernel 3, stride 1, bias=False) = Conv(padding=1)).

Tolerance: rel-L2 <= 1e-2 on y and dx (bf16 output rounding), <= 1e-2 on dW (f32 output of bf16 GEMMs).
"""
import pytest
import torch
import torch.nn.functional as F

from golden_util import rel_err
from long_context_biomedical_imaging_amd import kernels

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,S,Cin,Cout", [
    (2, (9, 10, 11), 32, 32),      # ragged volume, NT=1
    (1, (16, 16, 16), 96, 96),     # Swin-tiny stage-1 channels, NT=3
    (1, (7, 12, 5), 192, 96),      # UnetrUpBlock conv1 (2C -> C)
    (2, (9, 7, 13), 96, 192),      # ragged, two samples: the (3, 1, 3) weight-gradient tile (Cout, Cin % 96)
    (2, (6, 6, 6), 64, 128),       # NT=4
    (1, (8, 9, 10), 1, 96),        # encoder1 on the image: generic (Cin % 16 != 0) path
    (2, (1, 33, 47), 64, 32),      # 2-D (D = 1, 9 taps)
    (1, (1, 20, 24), 3, 64),       # 2-D generic
    (2, (1, 17, 19), 1, 32),       # 2-D Cin = 1: weight gradient as the im2col GEMM
    (1, (5, 6, 7), 2, 64),         # 3-D Cin = 2: the same
])
def test_conv3_parity(B, S, Cin, Cout):
    torch.manual_seed(0)
    nd = 2 if S[0] == 1 else 3
    shp = S[1:] if nd == 2 else S
    x = torch.randn(B, Cin, *shp).bfloat16().float()
    w = (torch.randn(Cout, Cin, *(3,) * nd) / (Cin * 27) ** 0.5).bfloat16().float()
    dy = torch.randn(B, Cout, *shp).bfloat16().float()
    conv = F.conv3d if nd == 3 else F.conv2d
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    yr = conv(xr, wr, padding=1)
    yr.backward(dy)
    xc = x.cuda().requires_grad_(True)
    wc = w.cuda().requires_grad_(True)
    y = kernels.conv3(xc, wc)
    assert y.shape == yr.shape and y.dtype == torch.bfloat16
    assert rel_err(y.float(), yr) < 1e-2
    y.backward(dy.cuda().bfloat16())
    assert rel_err(xc.grad.float(), xr.grad) < 1e-2
    assert rel_err(wc.grad, wr.grad) < 1e-2


@pytest.mark.parametrize("S,Cin,Cout", [((4, 4, 4), 768, 768), ((8, 8, 8), 384, 192), ((3, 5, 4), 256, 128)])
def test_conv3_split_k_small_volumes(S, Cin, Cout):
    """Small volumes (the 4^3 - 16^3 SwinUNETR stages) take the split-K form (lci_conv3_fwd_split: f32 partials of
    slab ranges, summed in split order): forward, data and weight gradients vs the fp32 conv on the host, and the
    split forward vs the unsplit kernel (LCI_CONV_SPLITK=0) within bf16 output rounding."""
    import os
    torch.manual_seed(2)
    assert kernels._lib.load().lci_conv3_fwd_splits(S[0] * S[1] * S[2], Cin, Cout, 3) > 1
    x = torch.randn(1, Cin, *S).bfloat16().float()
    w = (torch.randn(Cout, Cin, 3, 3, 3) / (Cin * 27) ** 0.5).bfloat16().float()
    dy = torch.randn(1, Cout, *S).bfloat16().float()
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    yr = F.conv3d(xr, wr, padding=1)
    yr.backward(dy)
    xc, wc = x.cuda().requires_grad_(True), w.cuda().requires_grad_(True)
    y = kernels.conv3(xc, wc)
    assert rel_err(y.float(), yr) < 1e-2
    y.backward(dy.cuda().bfloat16())
    assert rel_err(xc.grad.float(), xr.grad) < 1e-2
    assert rel_err(wc.grad, wr.grad) < 1e-2
    os.environ["LCI_CONV_SPLITK"] = "0"
    try:
        y1 = kernels.conv3(x.cuda(), w.cuda())
    finally:
        del os.environ["LCI_CONV_SPLITK"]
    assert rel_err(y.float(), y1.float()) < 4e-3


def test_conv3_large_vs_miopen():
    """Swin-tiny decoder1 shape at 64^3 (96 -> 96): against torch's (MIOpen) bf16 conv on the GPU."""
    torch.manual_seed(1)
    x = torch.randn(1, 96, 64, 64, 64, device="cuda").bfloat16()
    w = (torch.randn(96, 96, 3, 3, 3, device="cuda") / (96 * 27) ** 0.5)
    y = kernels.conv3(x, w)
    yr = F.conv3d(x.float(), w.bfloat16().float(), padding=1)
    assert rel_err(y.float(), yr) < 1e-2


@pytest.mark.parametrize("shape", [(2, 96, 9, 10, 11), (1, 64, 33, 47), (1, 1536, 3, 3, 3), (2, 32, 40, 3, 5)])
@pytest.mark.parametrize("act", [True, False])
def test_instance_norm_act_parity(shape, act):
    """lci_inorm (channels-last) vs torch InstanceNorm (affine=False, eps 1e-5) [+ LeakyReLU(0.01)] in fp32 on
    the same bf16 input; rel-L2 <= 1e-2 (bf16 output) forward, <= 2e-2 input gradient."""
    torch.manual_seed(0)
    x = (torch.randn(shape) * 3 + 0.5).bfloat16().float()
    dz = torch.randn(shape).bfloat16().float()
    xr = x.clone().requires_grad_(True)
    zr = F.instance_norm(xr, eps=1e-5)
    if act:
        zr = F.leaky_relu(zr, 0.01)
    zr.backward(dz)
    xc = x.cuda().bfloat16().requires_grad_(True)
    z = kernels.instance_norm_act(xc, act)
    assert z.shape == zr.shape and z.dtype == torch.bfloat16
    assert rel_err(z.float(), zr) < 1e-2
    z.backward(dz.cuda().bfloat16())
    assert rel_err(xc.grad.float(), xr.grad) < 2e-2


def _ref_resblock(blk, x):
    """MONAI-1.3 UnetResBlock forward in plain torch ops on the module's own weights (moved to x's device):
    conv-norm-lrelu-conv-norm (+ conv3-norm3 residual) -> add -> lrelu. On CPU in fp32 it is the oracle; on the
    GPU under autocast it is the reference's own bf16 path (MIOpen convs, torch instance_norm)."""
    nd = x.dim() - 2
    conv = F.conv3d if nd == 3 else F.conv2d
    dev = x.device
    w = lambda m: m.weight if m.weight.device == dev else m.weight.detach().float().to(dev)   # noqa: E731
    out = F.leaky_relu(F.instance_norm(conv(x, w(blk.conv1.conv), padding=1), eps=1e-5), 0.01)
    out = F.instance_norm(conv(out, w(blk.conv2.conv), padding=1), eps=1e-5)
    res = F.instance_norm(conv(x, w(blk.conv3.conv)), eps=1e-5) if blk.downsample else x
    return F.leaky_relu(out + res, 0.01)


@pytest.mark.parametrize("nd,S,cin,cout", [(3, (12, 10, 14), 64, 32), (3, (8, 8, 8), 96, 96), (2, (40, 36), 128, 64)])
def test_unet_resblock_fused_vs_torch(nd, S, cin, cout):
    """Decoder block on the HIP conv + inorm kernels (channels-last) vs the fp32 torch restatement on the same
    weights and bf16-rounded input. Bound: no worse than 1.5x the error of the reference's own bf16 autocast path
    (torch/MIOpen on the GPU) against the same fp32 oracle, and <= 3e-2 on the output."""
    from long_context_biomedical_imaging_amd.decoders import UnetResBlock
    torch.manual_seed(0)
    blk = UnetResBlock(nd, cin, cout, 3, 1).cuda()
    assert blk.fused
    x = torch.randn(2, cin, *S).bfloat16().float()
    dy = torch.randn(2, cout, *S)
    xr = x.clone().requires_grad_(True)
    yr = _ref_resblock(blk, xr)                       # fp32 CPU oracle
    yr.backward(dy)
    xt = x.cuda().requires_grad_(True)                # reference's bf16 autocast path on the GPU
    with torch.autocast("cuda", dtype=torch.bfloat16):
        yt = _ref_resblock(blk, xt)
    yt.float().backward(dy.cuda())
    gt = blk.conv1.conv.weight.grad.float().cpu()
    blk.zero_grad(set_to_none=True)
    xc = x.cuda().requires_grad_(True)                # this repo's fused HIP path
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = blk(xc)
    assert y.shape == yr.shape
    y.float().backward(dy.cuda())
    e_y, e_yt = rel_err(y.float(), yr), rel_err(yt.float(), yr)
    e_dx, e_dxt = rel_err(xc.grad.float(), xr.grad), rel_err(xt.grad.float(), xr.grad)
    assert e_y < 3e-2 and e_y <= max(1.5 * e_yt, 1e-2), (e_y, e_yt)
    assert e_dx <= max(1.5 * e_dxt, 1e-2), (e_dx, e_dxt)
    # conv1 weight gradient against an fp32 CPU replay with conv1.weight as the leaf (same relative bound)
    g = blk.conv1.conv.weight.grad.float().cpu()
    wr = torch.nn.Parameter(blk.conv1.conv.weight.detach().float().cpu())
    blk.conv1.conv.weight = wr
    _ref_resblock(blk, x.clone()).backward(dy)
    e_g, e_gt = rel_err(g, wr.grad), rel_err(gt, wr.grad)
    assert e_g <= max(1.5 * e_gt, 1e-2), (e_g, e_gt)


@pytest.mark.parametrize("Cout,Cin,nd", [(96, 192, 3), (64, 1, 3), (32, 3, 2), (130, 70, 3)])
def test_conv3_weight_pack(Cout, Cin, nd):
    """lci_conv3_pack_weight: the forward operand (Cout, T, Cin) and the flipped, transposed data-gradient operand
    (Cin_pad, T, Cout) equal the torch expressions they replace, bit for bit (one bf16 rounding of the f32 weight)."""
    torch.manual_seed(4)
    kd = 3 if nd == 3 else 1
    w = torch.randn(Cout, Cin, *(3,) * nd, device="cuda")
    sp = tuple(range(2, 2 + nd))
    ref0 = w.to(torch.bfloat16).permute(0, *sp, 1).reshape(Cout, kd * 9, Cin)
    assert torch.equal(kernels._conv3_pack(w, kd, 0, Cin), ref0)
    cp = -(-Cin // 32) * 32
    ref1 = w.to(torch.bfloat16).flip(sp).permute(1, *sp, 0).reshape(Cin, kd * 9, Cout)
    ref1 = torch.cat([ref1, ref1.new_zeros(cp - Cin, kd * 9, Cout)])
    assert torch.equal(kernels._conv3_pack(w, kd, 1, cp), ref1)


@pytest.mark.parametrize("nd,S,cin,cout", [(3, (12, 10, 14), 64, 32), (3, (8, 8, 8), 96, 96), (2, (40, 36), 128, 64)])
def test_unet_resblock_fused_tail_bit_exact(nd, S, cin, cout, monkeypatch):
    """lci_inorm_apply_res (norm2 [+ norm3] + residual add + LeakyReLU in one pass) against the unfused kernel +
    torch sequence it replaces: same bf16 roundings, so output and every gradient are bitwise equal (downsample
    residual = norm3(conv3(x)); identity residual = the bf16 channels-last block input)."""
    from long_context_biomedical_imaging_amd.decoders import UnetResBlock
    torch.manual_seed(3)
    blk = UnetResBlock(nd, cin, cout, 3, 1).cuda()
    x = torch.randn(2, cin, *S, device="cuda").bfloat16()
    x = x.to(memory_format=torch.channels_last_3d if nd == 3 else torch.channels_last)
    dy = torch.randn(2, cout, *S, device="cuda").bfloat16()
    outs = []
    for fused in (True, False):
        if not fused:
            monkeypatch.setattr(kernels, "inorm_add_lrelu", lambda *a: None)
        blk.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = blk(xi)
        y.backward(dy)
        outs.append((y.detach(), xi.grad, blk.conv1.conv.weight.grad, blk.conv2.conv.weight.grad))
    for name, a, b in zip(("y", "dx", "dW1", "dW2"), outs[0], outs[1]):
        assert torch.equal(a, b), name


@pytest.mark.parametrize("B,S,Cin,Cout", [
    (1, (32, 32, 32), 96, 96),     # C3 stage-2 channels, many 128-row steps per split
    (2, (9, 7, 13), 192, 96),      # ragged lines (gap rows mid-step), two samples, Cin % 96
    (1, (12, 11, 10), 64, 192),    # the (1, 3, 2) tile (Cin % 64)
    (1, (1, 70, 50), 96, 96),      # 2-D (9 taps)
])
def test_conv3_wgrad_dma_vs_register_staging(B, S, Cin, Cout, monkeypatch):
    """Weight gradient v6 (LDS-DMA staging, three buffers; the default for the (1, 3, WC) tiles) against v5 (register
    staging, LCI_WGRAD_DMA=0): the same MFMA sequence over the same staged rows, so bitwise equal; and against the
    fp64 product over the same bf16 operands (f32 accumulation bound)."""
    torch.manual_seed(3)
    kd = 1 if S[0] == 1 else 3
    x = torch.randn(B, *S, Cin, device="cuda").bfloat16()
    dy = torch.randn(B, *S, Cout, device="cuda").bfloat16()
    g6 = kernels.conv3_wgrad_cl(x, dy, kd)
    monkeypatch.setenv("LCI_WGRAD_DMA", "0")
    g5 = kernels.conv3_wgrad_cl(x, dy, kd)
    monkeypatch.delenv("LCI_WGRAD_DMA")
    assert torch.equal(g6, g5)
    nd = 2 if kd == 1 else 3
    xs = x.double().movedim(-1, 1)
    dys = dy.double().movedim(-1, 1)
    if nd == 2:
        xs, dys = xs[:, :, 0], dys[:, :, 0]
    wr = torch.zeros(Cout, Cin, *(3,) * nd, dtype=torch.float64, device="cuda", requires_grad=True)
    conv = F.conv3d if nd == 3 else F.conv2d
    (conv(xs, wr, padding=1) * dys).sum().backward()
    ref = wr.grad.reshape(g6.shape)
    err = (g6.double() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 1e-4 * scale + 1e-6, f"max err {err:.3e} (max |ref| {scale:.3e})"
